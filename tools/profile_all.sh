#!/bin/bash
# The round's profile set: configs[1] (MLP-284 fp32 B=1024), configs[4] on one GPU (PER + bf16,
# B=8192), configs[2] stress (4,84,84) B=256 and the reference HEAD net (2,27,5) B=256, each through
# tools/profile_round.sh.  WHICH selects a subset (default: all).
set -u
export ROUND_NAME=${ROUND_NAME:-round}
W=${WHICH:-"mlp c5 hyb84 hyb"}
for w in $W; do
  case $w in
    mlp)   NET=mlp B=1024 TAG= BENCH_ARGS="${EXTRA:-}" bash tools/profile_round.sh || exit $? ;;
    c5)    NET=mlp B=8192 TAG=_bf16 BENCH_ARGS="--algo PerDuelingDoubleDQNAgent --compute bf16 --batch 8192 ${EXTRA:-}" bash tools/profile_round.sh || exit $? ;;
    hyb84) NET=hybrid84 B=256 TAG= BENCH_ARGS="--net hybrid84 --batch 256 --steps 50 --warmup 5 ${EXTRA:-}" bash tools/profile_round.sh || exit $? ;;
    hyb)   NET=hybrid B=256 TAG= BENCH_ARGS="--net hybrid --batch 256 ${EXTRA:-}" bash tools/profile_round.sh || exit $? ;;
  esac
done
