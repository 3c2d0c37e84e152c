#!/bin/bash
# Build libdgn.so of a git revision into defect-gnn-cpp_amd/lib/libdgn_<tag>.so (A/B baselines):
#   bash tools/build_rev.sh <rev> <tag> [extra hipcc flags]
set -eo pipefail
REV=$1; TAG=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/dgn_wt_$TAG
rm -rf "$WT"
git -C "$ROOT" worktree add -f --detach "$WT" "$REV" > /dev/null
make -C "$WT" -j8 defect-gnn-cpp_amd/lib/libdgn.so HIPFLAGS_EXTRA="$*" > /dev/null
cp "$WT/defect-gnn-cpp_amd/lib/libdgn.so" "$ROOT/defect-gnn-cpp_amd/lib/libdgn_$TAG.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $ROOT/defect-gnn-cpp_amd/lib/libdgn_$TAG.so from $(git -C "$ROOT" rev-parse --short "$REV")"
