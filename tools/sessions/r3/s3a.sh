#!/usr/bin/env bash
# round 3, session 3: new GPU tests (K-split co-resident, config 2 exact path,
# config 4 at its stated size), then config 2 under a kernel trace (launch gaps)
set -u
R="$GRAFT_REPO_ROOT"; out=$R/gpurun_out/s3a; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "coresident or config2 or config4 or capi" > $out/newtests.log 2>&1 || { tail -40 $out/newtests.log; exit 1; }
tail -3 $out/newtests.log
timeout -k 10 120 python -u tools/configs_bench.py single > $out/single.log 2>&1 || { tail $out/single.log; exit 1; }
tail -2 $out/single.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof_single -o run --output-format csv -- python3 $R/tools/configs_bench.py single > $out/prof_single.log 2>&1 || { tail $out/prof_single.log; exit 1; }
ls -R $out/prof_single | head
