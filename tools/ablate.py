#!/usr/bin/env python3
"""Ablation builds of the flow kernel (development tool): each variant is
agnes_flow.hip with one text substitution (timing only: the results are wrong by
design), linked with the other engine objects into agnes_amd/_exp/lib_<name>.so.
Run on the GPU box with  AGNES_LIB=agnes_amd/_exp/lib_<name>.so python tools/kbench.py ...

usage: tools/ablate.py build   |   tools/ablate.py list"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from agnes_amd import build as B  # noqa: E402

EXP = os.path.join(ROOT, "agnes_amd", "_exp")
SRC = os.path.join(B.CSRC, "agnes_flow.hip")

# name -> list of (old, new) substitutions
VARIANTS = {
    "base": [],
    "nomulti": [("const bool multi = bk != 0ull;", "const bool multi = false; bk = 0;")],
    "nophase2": [("""                        uint32_t l = sv + sn > ta ? 1u : 0u;
                        l = sn > tn ? 2u : l;
                        l = sv > tv ? 3u : l;""", "                        uint32_t l = (sv ^ sn ^ (uint32_t)tv ^ (uint32_t)tn ^ (uint32_t)ta) & 3u;")],
    "nosm": [("if (ballot((x0 | x1) != 0u)) {", "if (false) {")],
    "noroles": [("if (SM) {\n                    uint32_t* const rA", "if (false) {\n                    uint32_t* const rA")],
    "novalid": [("all_ok = !ballot((actA && !okA) || (actB && !okB));", "all_ok = true; (void)okA; (void)okB;")],
    "memonly": [("                /* ---- K2 + K3: one pass per round present ---- */",
                 "                uint32_t c0 = w[0] ^ w[1] ^ w[2] ^ w[3] ^ nb0, c1 = w[4] ^ w[5] ^ w[6] ^ w[7] ^ nb1;\n"
                 "                if (false) {\n                /* ---- K2 + K3: one pass per round present ---- */"),
                ("                /* codes (deferred) */", "                }\n                /* codes (deferred) */"),
                ("                uint32_t c0 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv0 | (ts0c >> 3));",
                 "                c0 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv0 | (ts0c >> 3));"),
                ("                uint32_t c1 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv1 | (ts1c >> 3));",
                 "                c1 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv1 | (ts1c >> 3));")],
    "nont": [("global_load_lds_dwordx4 %1, %2 nt", "global_load_lds_dwordx4 %1, %2"),
             ("global_load_lds_dword %1, %2 nt", "global_load_lds_dword %1, %2")],
    "wpe4": [("__global__ __launch_bounds__(256) void flow(",
              "__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void flow(")],
    "k4fast": [("if (!ballot(inA || inB)) { /* no P1 or C inside any unit: whole-unit masks */",
                "if (true) { (void)inA; (void)inB;")],
    "k4norec": [("if (!crossedC && bC < 4) rk[R_C] = pos + (uint32_t)bC;", "(void)rk;"),
                ("if (!crossedP && p1ok && bP < 4) rk[R_P1] = pos + (uint32_t)bP;", "")],
    "k4nowrite": [("if (ballot((lk0 | lk1 | aC0 | aC1 | v0 | v1) != 0u)) {", "if (false) {")],
    "nostore": [("            if (dc_act == 2u) sstore8(a.codes + dc_at, o8, dc0, dc1);",
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
    for name, subs in VARIANTS.items():
        t = text
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
    if sys.argv[1:] == ["build"]:
        build()
    else:
        print(" ".join(VARIANTS))
