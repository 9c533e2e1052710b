#!/bin/bash
# PMC passes over batch-1 forwards (tools/batch1_trace.py): L2 hits / misses, HBM fetch bytes,
# L1 -> L2 read requests and L1 accesses, per serving conv launch (tools/convs_pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/convs_pmc
rm -rf $O; mkdir -p $O
i=0
for C in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o run -- python3 tools/batch1_trace.py > $O/p$i.log 2>&1 || { echo "pmc $C failed rc=$?"; tail -5 $O/p$i.log; exit 3; }
  echo "pmc $C ok"
done
python3 tools/convs_pmc_summary.py $O/p1 $O/p2 $O/p3 $O/p4
