#!/bin/bash
# round 6: section stamps of the shipped gi_gram and of the blocked-solve
# variant (lib/libqpb_gblk.so swapped in on the box copy only).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6j}; mkdir -p $O
echo "== stamps head" && timeout -k 10 300 python tools/gram_time.py > $O/gram_time_head.txt 2>&1 || { tail -5 $O/gram_time_head.txt; exit 1; }
tail -1 $O/gram_time_head.txt
cp embedded-qp-solver_amd/lib/libqpb_gblk.so embedded-qp-solver_amd/lib/libqpb.so
echo "== stamps gblk" && timeout -k 10 300 python tools/gram_time.py > $O/gram_time_gblk.txt 2>&1 || { tail -5 $O/gram_time_gblk.txt; exit 1; }
tail -1 $O/gram_time_gblk.txt
exit 0
