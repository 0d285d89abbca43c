#!/usr/bin/env bash
# A/B kernel variants: tools/ab.sh "<kbench args>" variant1.so variant2.so ...
# Interleaves 2 rounds over the variants; one kbench process per (round, variant).
args="$1"; shift
for round in 1 2; do
  for v in "$@"; do
    echo "## round $round variant $(basename "$v")"
    NERFHIP_LIB="$v" timeout -k 5 120 python tools/kbench.py $args --repeat 1 | grep rep || exit $?
  done
done
