#!/bin/bash
# Kernel + memory-copy trace of one-prepare commits on a 2-shard node engine.
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r04node1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o run -- \
  python3 $R/tools/gpu/node_one_prepare.py 120 2 > $O/run.log 2>&1 || exit 1
tail -2 $O/run.log
