#!/usr/bin/env bash
set -u
bash tools/ks_round.sh d || exit 1
bash tools/split_probe.sh || exit 1
