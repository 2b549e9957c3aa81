#!/usr/bin/env python3
"""Static instruction mix of the tally kernels (development tool).
usage: tools/isa_stats.py kernel.s [substring-of-mangled-name ...]"""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:] or [""]
for m in re.finditer(r"^(_ZN5agnes12tally_kernelI\w+):", s, re.M):
    n = m.group(1)
    if not any(p in n for p in pats):
        continue
    b = s.index(".Lfunc_end", m.end())
    ins = [l.strip() for l in s[m.end():b].split("\n") if l.startswith("\t") and l.strip()
           and not l.strip().startswith((".", ";"))]
    cnt = lambda *p: sum(1 for l in ins if l.startswith(p))
    print(n.split("tally_kernelI")[1][:22], "total", len(ins), "valu", cnt("v_"), "salu", cnt("s_"),
          "vmem", cnt("global_", "buffer_", "flat_"), "lds", cnt("ds_"),
          "readlane", cnt("v_readlane", "v_readfirstlane"), "writelane", cnt("v_writelane"),
          "dpp", sum(1 for l in ins if "row_" in l), "waitcnt", cnt("s_waitcnt"), "nop", cnt("s_nop"))
