#!/bin/bash
# rocprofv3 evidence for round 3: the headline leg's kernel trace + stats (tools/gpu/profile.sh kt),
# the adversarial C3's, and FETCH_SIZE / WRITE_SIZE passes of device-resident C2 passes.
cd "$GRAFT_REPO_ROOT" || exit 1
for m in kt c3h dfetch dwrite; do
  bash tools/gpu/profile.sh $m > gpurun_out/prof_$m.txt 2>&1
  echo "$m rc=$?"
done
exit 0
