"""restir_amd -- MI355X-native ReSTIR DI renderer (host-side Python binding of librestir_amd.so).

The hot path (BVH build + traversal, the ReSTIR passes) is hand-written HIP for gfx950 behind the
C ABI in include/restir_c.h; this package only marshals scenes/parameters and drives frames.
"""
from . import params, scenes  # noqa: F401
from .params import FrameParams, default_params, metric_params, c3_params  # noqa: F401
from .renderer import Renderer, Scene, RestirError, load_library, LIB_PATH, EXPORTED_SYMBOLS  # noqa: F401
from .denoise import Denoiser, check_weights  # noqa: F401
