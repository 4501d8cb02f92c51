#!/bin/bash
# Interleaved A/B of the Fisher pipeline (GPU box, repo root): libgsr.so vs splatam_amd/_diag/libgsr_<tag>.so for each tag in $TAGS
for r in 1 2; do for t in base ${TAGS:-f4 f0}; do L=splatam_amd/libgsr.so; [ $t != base ] && L=splatam_amd/_diag/libgsr_$t.so; echo -n "$t "; GSR_LIB=$L timeout -k 10 120 python tools/fisher_bench.py --launches 20 2>/dev/null | tail -1; done; done
