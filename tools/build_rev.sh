#!/bin/bash
# Build libgsplat_mi355x.so of git revision REV (its csrc/ and include/) into OUT, for same-box
# A/B runs (GSPLAT_MI355X_LIB=OUT).  Usage: tools/build_rev.sh REV OUT
set -e
rev=$1; out=$(realpath -m "$2")
d=$(mktemp -d /tmp/build_rev.XXXX)
mkdir -p "$d/gaussctrl_exp_amd" "$d/include"
git archive "$rev" gaussctrl_exp_amd/csrc include | tar -x -C "$d"
make -s -C "$d/gaussctrl_exp_amd/csrc" -j8 OUT="$out" "$out"
rm -rf "$d"
