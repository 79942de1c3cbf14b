#!/bin/bash
# Build a committed revision next to the working tree for same-box A/B runs:
#   tools/mk_ab_old.sh <rev>  ->  ab_old/{bench.py, vision-instance-seg_amd/} (git-ignored,
#   travels with gpurun); run `python3 ab_old/bench.py ...` beside `python3 bench.py ...`.
set -e
rev=${1:-HEAD}
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d /tmp/abold.XXXX)
git -C "$root" worktree add --detach "$tmp/t" "$rev" >/dev/null
make -s -C "$tmp/t/vision-instance-seg_amd" -j8 >/dev/null
rm -rf "$root/ab_old"
mkdir -p "$root/ab_old"
cp "$tmp/t/bench.py" "$root/ab_old/"
cp -r "$tmp/t/vision-instance-seg_amd" "$root/ab_old/"
rm -rf "$root/ab_old/vision-instance-seg_amd/build"
git -C "$root" worktree remove --force "$tmp/t"
rm -rf "$tmp"
echo "ab_old = $(git -C "$root" rev-parse --short "$rev")"
