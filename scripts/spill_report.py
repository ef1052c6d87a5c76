"""Diagnostic: where a kernel's scratch (spill) instructions sit -- compiles csrc/restir_capi.hip to gfx950
assembly with the Makefile's flags and prints, per kernel, scratch loads/stores in total and inside
loops, with the innermost enclosing loop's length in instructions (a spill in a walk loop costs per
node step, one in the candidate loop per candidate).  Usage: python scripts/spill_report.py [substr ...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "restir-embree_amd")


def flags():
    mk = open(os.path.join(PKG, "Makefile")).read()
    f = re.search(r"HIPFLAGS \?=(.*?)\n(?!\s)", mk, re.S).group(1).replace("\\\n", " ").replace("$(ARCH)", "gfx950")
    out = [x for x in f.split() if not x.startswith("-W")]
    for extra in os.environ.get("EXTRA_FLAGS", "").split():   # e.g. EXTRA_FLAGS=-DRS_INITIAL_WAVES_LANE=6
        name = extra.split("=")[0]
        out = [x for x in out if x.split("=")[0] != name] + [extra]
    return out


def main():
    want = sys.argv[1:] or ["k_gbuffer_initial", "k_spatial", "k_temporal"]
    out = "/tmp/restir_capi.s"
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags(), "-w", "--cuda-device-only", "-S", "-o", out,
                           os.path.join(PKG, "csrc", "restir_capi.hip")], cwd=PKG)
    s = open(out).read()
    for m in re.finditer(r"^(_Z\S+):(?:\s*;.*)?$", s, re.M):
        name = m.group(1)
        if not any(w in name for w in want):
            continue
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end].splitlines()
        labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
        loops = []
        for k, l in enumerate(body):
            b = re.search(r"s_(?:cbranch_\w+|branch) (\.LBB\d+_\d+)", l)
            if b and b.group(1) in labels and labels[b.group(1)] < k:
                loops.append((labels[b.group(1)], k))
        ops = [k for k, l in enumerate(body) if "scratch_load" in l or "scratch_store" in l]
        inner = sorted(min(hi - lo for lo, hi in loops if lo <= k <= hi) for k in ops
                       if any(lo <= k <= hi for lo, hi in loops))
        vg = re.search(r"\.vgpr_count:\s+(\d+)", s[end:end + 200000])
        print(f"{name[:64]}: {len(ops)} scratch ops, {len(inner)} in loops (innermost loop lengths {inner[:16]})")


if __name__ == "__main__":
    main()
