#!/bin/bash
# Export git revision REV's whole tree into DIR and build its libraries there, for same-box A/B
# runs of an earlier round's own bench.py (its Python and C-ABI together: the ABI changes
# between rounds, so a library alone cannot be swapped in).  Usage: tools/build_tree.sh REV DIR
set -e
rev=$1; dir=$2
rm -rf "$dir"; mkdir -p "$dir"
git archive "$rev" | tar -x -C "$dir"
rm -rf "$dir/profiles" "$dir/tests/golden/harness_"* 2>/dev/null || true
make -s -C "$dir/gaussctrl_exp_amd/csrc" -j8 > /dev/null
