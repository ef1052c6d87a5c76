"""Per-frame parameter snapshot (``rs_frame_params`` in include/restir_c.h).

The reference keeps every ReSTIR knob in mutable static globals edited live by ImGui
(pg/ReSTIRIntegrator.cpp:13-35, written at :37-87) plus ReSTIR's private RenderParams
(pg/RenderParams.h:5-17).  Here they are a POD struct passed by value per frame, which removes the
reference's UI/render race.  Defaults are the reference's defaults except ``use_skybox`` (the
reference default is true, but its sky HDR is a missing blob, so miss pixels use bg_color).
"""
from __future__ import annotations

import ctypes

# ReSTIRIntegrator::SpatialWeightCalculation (pg/ReSTIRIntegrator.h:19-25)
CONSTANT, CONSTANT_DEBIAS_CONTRIB, CONSTANT_DEBIAS_Z_TERM, BALANCE_HEURISTIC, PAIRWISE_MIS = range(5)
MIS_NAMES = {"constant": CONSTANT, "debias_contrib": CONSTANT_DEBIAS_CONTRIB, "debias_z": CONSTANT_DEBIAS_Z_TERM,
             "balance": BALANCE_HEURISTIC, "pairwise": PAIRWISE_MIS}


class FrameParams(ctypes.Structure):
    _fields_ = [
        ("m_area", ctypes.c_int32),               # M_Area            (:13)
        ("m_brdf", ctypes.c_int32),               # M_Brdf            (:14)
        ("spatial_neighbors", ctypes.c_int32),    # spatialReuseNeighborCount (:16)
        ("spatial_passes", ctypes.c_int32),       # spatialPassCount  (:17)
        ("confidence_cap", ctypes.c_int32),       # confidenceCap     (:18)
        ("spatial_radius", ctypes.c_float),       # spatialReuseRadius (:19)
        ("min_normal_similarity", ctypes.c_float),  # (:20)
        ("max_depth_difference", ctypes.c_float),   # (:21)
        ("do_spatial", ctypes.c_int32),           # doSpatialReuse    (:24)
        ("do_temporal", ctypes.c_int32),          # doTemporalReuse   (:25)
        ("do_visibility_pass", ctypes.c_int32),   # doVisibilityPass  (:27)
        ("reject_dissimilar", ctypes.c_int32),    # rejectDissimilarNeighbors (:29)
        ("spatial_mis", ctypes.c_int32),          # spatialWeightCalc (:33)
        ("use_skybox", ctypes.c_int32),           # RenderParams::useSkybox
        ("bg_color", ctypes.c_float * 3),         # RenderParams::bgColor
        ("tnear_offset", ctypes.c_float),         # RenderParams::tnearOffset
        ("tfar_offset", ctypes.c_float),          # RenderParams::tfarOffset
        ("normal_offset", ctypes.c_float),        # RenderParams::normalOffset
        ("seed", ctypes.c_uint32),                # counter-RNG base seed (reference: mt19937{123})
        ("debug_reprojection", ctypes.c_int32),   # debugReprojection (:30, :647-689)
    ]


def default_params(**kw) -> FrameParams:
    p = FrameParams()
    p.m_area, p.m_brdf = 1, 1
    p.spatial_neighbors, p.spatial_passes, p.confidence_cap = 5, 1, 20
    p.spatial_radius, p.min_normal_similarity, p.max_depth_difference = 30.0, 0.85, 0.2
    p.do_spatial = p.do_temporal = p.do_visibility_pass = p.reject_dissimilar = 0
    p.spatial_mis = CONSTANT
    p.use_skybox = 0
    p.bg_color[0] = p.bg_color[1] = p.bg_color[2] = 0.5
    p.tnear_offset, p.tfar_offset, p.normal_offset = 0.01, 0.001, 0.001
    p.seed = 123
    p.debug_reprojection = 0
    for k, v in kw.items():
        if k == "bg_color":
            for i in range(3):
                p.bg_color[i] = v[i]
        elif k == "spatial_mis" and isinstance(v, str):
            p.spatial_mis = MIS_NAMES[v]
        else:
            if not hasattr(p, k):
                raise AttributeError(k)
            setattr(p, k, v)
    return p


def metric_params(**kw) -> FrameParams:
    """BASELINE.json metric point / C2: A=32 area candidates, B=1 BRDF candidate, spatial k=4,
    P=1, R=30, CONSTANT MIS, cap 20, temporal off, visibility pass off."""
    base = dict(m_area=32, m_brdf=1, spatial_neighbors=4, spatial_passes=1, spatial_radius=30.0,
                do_spatial=1, do_temporal=0, spatial_mis=CONSTANT, confidence_cap=20)
    base.update(kw)
    return default_params(**base)


def c3_params(**kw) -> FrameParams:
    """C3/C5: metric point + temporal reuse on."""
    base = dict(do_temporal=1)
    base.update(kw)
    return metric_params(**base)
