#!/usr/bin/env python3
"""Ablation builds of the flow kernel (development tool): each variant is
agnes_flow.hip with one text substitution (timing only: the results are wrong by
design), linked with the other engine objects into agnes_amd/_exp/lib_<name>.so.
Run on the GPU box with  python tools/withlib.py agnes_amd/_exp/lib_<name>.so tools/kbench.py ...

usage: tools/ablate.py build   |   tools/ablate.py list"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agnes_amd import build as B  # noqa: E402

EXP = os.path.join(ROOT, "agnes_amd", "_exp")
SRC = os.path.join(B.CSRC, "agnes_flow.hip")

import re  # noqa: E402


def _lane_now(t):
    """per-lane offsets and lane ids in the batch-level code recomputed where used
    (an asm lane id LICM cannot hoist): fewer loop-carried VGPRs"""
    helper = ("__device__ __forceinline__ uint32_t lane_now() {\n    uint32_t l;\n"
              "    asm volatile(\"v_mbcnt_lo_u32_b32 %0, -1, 0\\n\\tv_mbcnt_hi_u32_b32 %0, -1, %0\" : \"=v\"(l));\n"
              "    return l;\n}\n")
    t = t.replace("__device__ __forceinline__ uint64_t u64of(", helper + "__device__ __forceinline__ uint64_t u64of(")

    def sub_in(t, a, b, first_brace=True):
        i = t.index(a)
        j = t.index(b, i)
        blk = re.sub(r"\blane\b", "lane_now()", t[i:j])
        return t[:i] + blk + t[j:]
    t = sub_in(t, "    auto finalize = [&]", "    Hdr H, N;")
    t = sub_in(t, "                if (rc == 0u && lane < m) { /* instance records */", "                if (SM && smf) {")
    t = sub_in(t, "                if (SM && smf) { /* the State machine", "                /* the next batch")
    t = t.replace("    const uint32_t o32 = 32u * lane, o16 = 16u * lane, o8 = 8u * lane, o4 = 4u * lane;",
                  "#define o32 (32u * lane_now())\n#define o16 (16u * lane_now())\n#define o8 (8u * lane_now())\n"
                  "#define o4 (4u * lane_now())")
    return t


def _w(n):
    return [("amdgpu_waves_per_eu(3)", f"amdgpu_waves_per_eu({n})")]


# name -> list of (old, new) substitutions, or a function of the text
VARIANTS = {
    "base": [],
    "w4": _w(4),
    "lanenow": _lane_now,
    "lanenow_w4": lambda t: _lane_now(t).replace("amdgpu_waves_per_eu(3)", "amdgpu_waves_per_eu(4)"),
    "nosm": [("if (ballot((x0 | x1) != 0u)) {", "if (false) {")],
    "noroles": [("if (SM) {\n                    uint32_t* const rA", "if (false) {\n                    uint32_t* const rA")],
    "k4nowrite2": [("if (ballot((lk0 | lk1 | aC0 | aC1 | v0 | v1) != 0u)) {", "if (false) {")],
    "k4nomsg": [("                        c0 |= unit(x0,", "                        (void)unit(x0,"),
                ("                        c1 |= unit(x1,", "                        (void)unit(x1,")],
    "nophase2": [("""                        uint32_t l = sv + sn > ta ? 1u : 0u;
                        l = sn > tn ? 2u : l;
                        l = sv > tv ? 3u : l;""", "                        uint32_t l = (sv ^ sn ^ (uint32_t)tv ^ (uint32_t)tn ^ (uint32_t)ta) & 3u;")],
    "k4nowrite": [("if (ballot((lk0 | lk1 | aC0 | aC1 | v0 | v1) != 0u)) {", "if (false) {")],
    "k4noval": [("                            if (v0) { /* valid (:198, :202): the last candidate */", "                            if (false) {"),
                ("                            if (v1) {\n                                const uint32_t b = (31u", "                            if (false) {\n                                const uint32_t b = (31u")],
    "k4fast": [("if (!ballot(inA || inB)) { /* no P1 or C inside any unit: whole-unit masks */",
                "if (true) { (void)inA; (void)inB;")],
    "k4norec": [("if (!crossedC && bC < 4) rk[R_C] = pos + (uint32_t)bC;", "(void)rk;"),
                ("if (!crossedP && p1ok && bP < 4) rk[R_P1] = pos + (uint32_t)bP;", "")],
    "nocf": [("""                    if (SM) {
                        /* unit A: its running sums""", """                    if (false) {
                        /* unit A: its running sums""")],
    "nowo": [("            reinterpret_cast<uint4*>(a.states + pend_s0)[lane] = *reinterpret_cast<const uint4*>(sbp + o16);",
              "            (void)sbp;")],
    "noreq": [("                    if (pend_stage == 2u) writeout();\n                    else request();",
               "                    if (pend_stage == 2u) writeout();\n                    else pend_stage = 2;")],
    "nodst": [("        glds16(reinterpret_cast<const unsigned char*>(st_in + h.s0) + 16u * (lane < 4u * m ? lane : 0u),\n"
               "               sb + par * (FB * 64u));", "        (void)par;")],
    "nostore": [("            if (dc_act == 3u) sstore8(a.codes + dc_at, o8, dc0, dc1);",
                 "            if (dc_act == 7u) sstore8(a.codes + dc_at, o8, dc0, dc1);")],
}


def objs():
    os.makedirs(EXP, exist_ok=True)
    out = []
    for s in B.SOURCES:
        if s == "agnes_flow.hip":
            continue
        o = os.path.join(EXP, s + ".o")
        if not os.path.exists(o) or os.path.getmtime(o) < os.path.getmtime(os.path.join(B.CSRC, s)):
            subprocess.run([B.HIPCC] + [f for f in B.FLAGS if f != "-shared"] + ["-c", "-o", o, os.path.join(B.CSRC, s)],
                           check=True, cwd=B.CSRC)
        out.append(o)
    return out


def build():
    base = objs()
    text = open(SRC).read()
    only = sys.argv[2:]
    for name, subs in VARIANTS.items():
        if only and name not in only:
            continue
        t = text
        if callable(subs):
            t = subs(t)
        else:
            for old, new in subs:
                assert old in t, (name, old)
                t = t.replace(old, new)
        src = os.path.join(B.CSRC, f"_abl_{name}.hip")
        open(src, "w").write(t)
        try:
            o = os.path.join(EXP, f"flow_{name}.o")
            subprocess.run([B.HIPCC] + [f for f in B.FLAGS if f != "-shared"] + ["-w", "-c", "-o", o, src], check=True, cwd=B.CSRC)
            subprocess.run([B.HIPCC] + B.FLAGS + ["-o", os.path.join(EXP, f"lib_{name}.so"), o] + base, check=True)
        finally:
            os.remove(src)
        print("built", name)


if __name__ == "__main__":
    if sys.argv[1:2] == ["build"]:
        build()
    else:
        print(" ".join(VARIANTS))
