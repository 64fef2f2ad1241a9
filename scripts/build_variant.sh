#!/bin/bash
# Build an A/B variant of the library: bash scripts/build_variant.sh NAME "-DFLAG=..." -> okvis2-x_amd/lib_NAME.so
set -e
cd "$(dirname "$0")/.."
make -s -C okvis2-x_amd -j8 BUILD=build_$1 LIB=lib_$1.so OPT="-O3 $2" lib_$1.so
