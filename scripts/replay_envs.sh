#!/bin/bash
# Replay one fuzz seed under several engine switches (one process each).
# usage: scripts/replay_envs.sh <seed> "<ENV=v ...>" ...
set -u
SEED=$1; shift
OUT=gpurun_out/fuzz
mkdir -p $OUT
for v in "$@"; do
  e=$v; [ "$v" = "none" ] && e=""
  echo "=== $v"
  env $e timeout -k 10 120 python3 -u scripts/fuzz_replay.py $SEED > $OUT/replay_${SEED}_$(echo "$v" | tr '= ' '__').log 2>&1 || { echo "rc=$?"; tail -5 $OUT/replay_${SEED}_$(echo "$v" | tr '= ' '__').log; exit 1; }
  tail -12 $OUT/replay_${SEED}_$(echo "$v" | tr '= ' '__').log
done
