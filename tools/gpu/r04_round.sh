#!/bin/bash
# One measurement call: write-back tests + replica path, validate A/B, C3h A/B.
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R" || exit 1
AB="r3val noearly cur" bash tools/gpu/r04_wb.sh || exit 1
AB_VARIANTS="norefresh cur" bash tools/gpu/r04_c3h_ab.sh
