#!/bin/bash
# Round 5, session 4: digit-sort pass variants timed by tools/sort_check big (2^28 MSM-like pairs,
# 16 and 19 key bits): base (C-form bitop ranking), lb4 / lb8 (4 / 8 predecessors' status words
# in flight in the look-back), nolb (TIMING PROBE, wrong order: no look-back), oldrank (round 4).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
: > $O/sort_variants.txt
for v in base lb4 lb8 oldrank nolb; do
  timeout -k 10 180 variants/sort_check_$v big > $O/sort_check_$v.txt 2>&1 || { tail -3 $O/sort_check_$v.txt; exit 1; }
  echo "$v ok=$(grep -c '"ok":1' $O/sort_check_$v.txt) bad=$(grep -c '"ok":0' $O/sort_check_$v.txt) $(grep '"time"' $O/sort_check_$v.txt | tr '\n' ' ')" | tee -a $O/sort_variants.txt
done
