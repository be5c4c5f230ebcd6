#!/bin/bash
# round 6: the LDS tie kernel's heap capacity (and with it the rows per CU) on the 10 k whole-ms graph
set -o pipefail
O=gpurun_out/r06_tiehc
mkdir -p $O
for hc in default 1024 600 400; do
  if [ $hc = default ]; then E=X=1; else E=SHD_PC_TIE_HC=$hc; fi
  env $E timeout -k 10 300 python3 -u scripts/r06/apsp_ties.py > $O/apsp_$hc.log 2>&1 || exit 2
  echo "$hc $(tail -n 1 $O/apsp_$hc.log)" >> $O/summary.txt
done
