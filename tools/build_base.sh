#!/bin/bash
# Container-side: build the library of a git revision (default HEAD) into
# se3-icp_amd/lib_<name>/libse3icp.so for same-box A/B runs against the working tree
# (tools/ab_pair.sh base se3-icp_amd/lib_base/libse3icp.so new se3-icp_amd/lib/libse3icp.so).
# Usage: tools/build_base.sh [rev] [name]
REV=${1:-HEAD}; NAME=${2:-base}
cd "$(dirname "$0")/.." || exit 1
WT=/tmp/se3icp_wt_$NAME
rm -rf "$WT"; git worktree prune
git worktree add --detach "$WT" "$REV" >/dev/null || exit 1
make -s -j8 -C "$WT/se3-icp_amd" lib/libse3icp.so || exit 1
mkdir -p "se3-icp_amd/lib_$NAME"
cp "$WT/se3-icp_amd/lib/libse3icp.so" "se3-icp_amd/lib_$NAME/libse3icp.so"
git worktree remove --force "$WT"
echo "se3-icp_amd/lib_$NAME/libse3icp.so <- $(git rev-parse --short "$REV")"
