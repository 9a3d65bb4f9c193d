#!/bin/bash
# Kernel trace + SQ counters of the cold-key sort, block-cooperative (W=0)
# vs wave-independent (W=1) variant (diagnostic).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 0 1; do
  echo "=== LDE_COLD_SORT_W=$w"
  LDE_COLD_SORT_W=$w bash tools/quick_prof.sh || exit 1
  LDE_COLD_SORT_W=$w bash tools/quick_pmc.sh | grep -E "k_cold|k_sieve " || exit 1
  LDE_COLD_SORT_W=$w CNT="FETCH_SIZE" bash tools/quick_pmc.sh | grep -E "k_cold" || exit 1
  LDE_COLD_SORT_W=$w CNT="WRITE_SIZE" bash tools/quick_pmc.sh | grep -E "k_cold" || exit 1
done
