#!/bin/bash
# P = 4 scan (Q <= 16): 8 / 12 records in flight per wave (var_pf2 / var_pf3)
# against 4, now that its LDS reads are conflict-free.  Parity on the scan
# tests, then Q = 16 alternated.
set -o pipefail
bash tools/gpu_scan_ab.sh 16 main pf2 pf3 main pf2 pf3
