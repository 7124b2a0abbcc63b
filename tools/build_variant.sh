#!/bin/bash
# Build libkplace.so of git revision $1 (or "WORKTREE" = the working tree) into
# kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/$2.so for tools/ab_libs.sh.
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
mkdir -p "$OUT"
if [ "$1" = WORKTREE ]; then
  make -s -C "$REPO/kubernetes-native-distributed-ai-job-scheduler_amd" -j8 >/dev/null
  cp "$REPO/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so" "$OUT/$2.so"
else
  WT=$(mktemp -d /tmp/kpwt.XXXX)
  git -C "$REPO" worktree add -q --detach "$WT" "$1"
  make -s -C "$WT/kubernetes-native-distributed-ai-job-scheduler_amd" -j8 >/dev/null
  cp "$WT/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so" "$OUT/$2.so"
  git -C "$REPO" worktree remove --force "$WT"
fi
echo "built $OUT/$2.so"
