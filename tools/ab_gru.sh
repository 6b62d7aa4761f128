#!/bin/bash
# tools/exp_gru2.py on library variants built by tools/ab_build.sh (build/ab_<name>.so), two rounds:
#   bash tools/ab_gru.sh base variant1 ...
set -e
for r in 1 2; do for v in "$@"; do echo -n "$v "; DDSP_HIP_LIB=build/ab_$v.so timeout -k 10 120 python tools/exp_gru2.py 2>/dev/null; done; done
