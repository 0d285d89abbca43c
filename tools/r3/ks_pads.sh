#!/usr/bin/env bash
# K-split co-residency: does the failure depend on the workgroup's LDS allocation size?
# forward-only compile-time kernel (v_ksmodes) and the shipped runtime-mode kernel at several dynamic-LDS pads
set -u
out=gpurun_out/ks_pads; mkdir -p $out
export KS_CASES="256,2,16384,0"
for lib in ksmodes shipped; do
  for pad in 0 16 256 512 1024 1280 2048; do
    if [ $lib = shipped ]; then unset NERFHIP_LIB; else export NERFHIP_LIB=build/variants/v_$lib.so; fi
    KS_PADS=$pad timeout -k 10 120 python -u tools/r3/ks_probe.py ${lib}_pad$pad 2 > $out/${lib}_$pad.jsonl 2> $out/${lib}_$pad.err || { echo "$lib $pad failed"; tail -3 $out/${lib}_$pad.err; exit 1; }
    python3 -c "
import json
for l in open('$out/${lib}_$pad.jsonl'):
    r=json.loads(l); print(r['tag'],r['N'],r['rep'],'bad_blocks',r['bad_blocks'],'max_err %.2e'%r['max_err'], r.get('first_blocks','')[:6] if r.get('first_blocks') else '')"
  done
done
