#!/bin/bash
# Build libskp.so from a git revision (default HEAD) into OUT (default stablekeypoints_amd/libskp_base.so),
# for same-box A/B runs against the working tree via SKP_LIB=... (dev tool).
set -e
REV=${1:-HEAD}
OUT=${2:-stablekeypoints_amd/libskp_base.so}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/skp_variant_$$
rm -rf $W && mkdir -p $W
git -C $ROOT archive $REV stablekeypoints_amd/csrc include | tar -x -C $W
make -C $W/stablekeypoints_amd/csrc -j8 >/dev/null
cp $W/stablekeypoints_amd/libskp.so $ROOT/$OUT
rm -rf $W
echo "built $REV -> $OUT"
