#!/usr/bin/env bash
# K-split co-residency probe on the shipped library and the compile-time-mode variant
set -u
out=gpurun_out/ks_probe; mkdir -p $out
timeout -k 10 300 python -u tools/r3/ks_probe.py shipped 2 > $out/shipped.jsonl 2> $out/shipped.err || { tail $out/shipped.err; exit 1; }
NERFHIP_LIB=build/variants/v_ksmodes.so timeout -k 10 300 python -u tools/r3/ks_probe.py ksmodes 3 > $out/ksmodes.jsonl 2> $out/ksmodes.err || { tail $out/ksmodes.err; exit 1; }
cut -c1-260 $out/shipped.jsonl $out/ksmodes.jsonl
