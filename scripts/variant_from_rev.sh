#!/bin/bash
# Build libpv.so from a git revision into phase-vocoder_amd/build/variants/libpv_<name>.so
# (A/B against the working tree on the same GPU box: scripts/ab.sh <name>).
# usage: bash scripts/variant_from_rev.sh <rev> <name> [extra DEFS]
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2; defs=${3:-}
tmp=$(mktemp -d)
git archive "$rev" phase-vocoder_amd/csrc include | tar -x -C "$tmp"
out=$PWD/phase-vocoder_amd/build/variants
mkdir -p "$out"
make -C "$tmp/phase-vocoder_amd/csrc" variant NAME="$name" DEFS="$defs" -j8 > /dev/null
cp "$tmp/phase-vocoder_amd/build/variants/libpv_$name.so" "$out/"
rm -rf "$tmp"
echo "built $out/libpv_$name.so from $rev"
