#!/bin/bash
# round-5 GPU call B: the queue-tail / fast-start A/B (c3shard, c3, c2, c3w) and the flow timeline
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r5
timeout -k 10 300 python3 tools/flowdiag.py agnes_amd/_exp/lib_diag.so c3shard c3 c2 > gpurun_out/r5/flowdiag_t.jsonl 2> gpurun_out/r5/flowdiag_t.err || { tail -20 gpurun_out/r5/flowdiag_t.err; exit 1; }
cut -c1-420 gpurun_out/r5/flowdiag_t.jsonl
LIBS="new=- slow0=agnes_amd/_exp/lib_slow0.so tail0=agnes_amd/_exp/lib_tail0.so t512=agnes_amd/_exp/lib_t512.so" CFGS="c3shard c3 c2 c3w" REPS=2 bash tools/abn.sh
