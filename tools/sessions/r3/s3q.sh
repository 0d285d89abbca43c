#!/usr/bin/env bash
# K-split layout, round 2: K-split rows only on split-K groups (fused epilogue back to xoff)
set -u
R="$GRAFT_REPO_ROOT"
export SUFFIX=${SUFFIX:-q}; bash $R/tools/r3/s3o.sh && bash $R/tools/r3/s3p.sh
