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


def cfg(body):
    """Basic blocks of one kernel's assembly: [(first line, end line)] in layout order, and successor lists."""
    starts = [0]
    for k, l in enumerate(body):
        t = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", t) or t.startswith("; %bb."):
            starts.append(k)
        elif re.match(r"s_(cbranch_\w+|branch|endpgm|setpc_b64)\b", t):
            starts.append(k + 1)
    starts = sorted(set(x for x in starts if x < len(body)))
    order = [(a, b) for a, b in zip(starts, starts[1:] + [len(body)])]
    label_block = {}
    for bi, (a, b) in enumerate(order):
        for k in range(a, b):
            m = re.match(r"^(\.LBB\d+_\d+):", body[k].strip())
            if m:
                label_block[m.group(1)] = bi
    succ = []
    for bi, (a, b) in enumerate(order):
        last = ""
        for k in range(b - 1, a - 1, -1):
            t = body[k].strip()
            if t and not t.startswith((";", ".")):
                last = t
                break
        out = []
        m = re.match(r"s_(cbranch_\w+|branch) (\.LBB\d+_\d+)", last)
        if m and m.group(2) in label_block:
            out.append(label_block[m.group(2)])
        if not (last.startswith("s_branch") or last.startswith("s_endpgm") or last.startswith("s_setpc")):
            if bi + 1 < len(order):
                out.append(bi + 1)
        succ.append(out)
    return succ, order


def natural_loops(succ, order):
    """Natural loops (back edge u -> h with h dominating u): [(set of blocks, size in lines)]."""
    n = len(succ)
    pred = [[] for _ in range(n)]
    for u, vs in enumerate(succ):
        for v in vs:
            pred[v].append(u)
    full = set(range(n))
    dom = [full.copy() for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for v in range(1, n):
            ps = [dom[p] for p in pred[v]]
            nd = (set.intersection(*ps) if ps else set()) | {v}
            if nd != dom[v]:
                dom[v] = nd
                changed = True
    loops = []
    for u in range(n):
        for h in succ[u]:
            if h in dom[u]:
                body, work = {h, u}, ([u] if u != h else [])
                while work:
                    x = work.pop()
                    for p in pred[x]:
                        if p not in body:
                            body.add(p)
                            work.append(p)
                loops.append((body, sum(order[b][1] - order[b][0] for b in body)))
    return loops


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
        blocks, order = cfg(body)
        loops = natural_loops(blocks, order)
        ops = [k for k, l in enumerate(body) if "scratch_load" in l or "scratch_store" in l]
        owner = {}
        for bi, (lo, hi) in enumerate(order):
            for k in range(lo, hi):
                owner[k] = bi
        inner = []
        for k in ops:
            sizes = [sz for body_set, sz in loops if owner.get(k) in body_set]
            if sizes:
                inner.append(min(sizes))
        inner.sort()
        hist = {}
        for sz in inner:
            hist[sz] = hist.get(sz, 0) + 1
        print(f"{name[:64]}: {len(ops)} scratch ops, {len(inner)} in loops (innermost loop length: ops "
              f"{dict(sorted(hist.items()))})")


if __name__ == "__main__":
    main()
