#!/bin/bash
# Build an A/B variant of libskp.so with extra compile flags: tools/build_variant.sh NAME "-DFOO=1"
# -> build/var_NAME/libskp.so (use with SKP_LIB=build/var_NAME/libskp.so)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C $ROOT/stablekeypoints_amd/csrc -j8 OBJDIR=$ROOT/build/var_$1/obj LIB=$ROOT/build/var_$1/libskp.so EXTRA="$2"
