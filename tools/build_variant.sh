#!/bin/bash
# Builds an experiment variant of the product library: build/xp/libblt_bpe_NAME.so (objects in
# build/exp, which no GPU call ships) with extra
# compile flags (e.g. -DBLT_PAIRW=1).  Run tests or bench against it with BLT_LIB_PATH.
#   tools/build_variant.sh pw "-DBLT_PAIRW=1"
# KFLAGS (environment): extra flags for the kernel source only (e.g. -mllvm scheduler options)
# KSRC (environment): an alternative kernel source (a variant kept outside the product tree)
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
HF="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
mkdir -p "$R/build/exp"
$HIPCC $HF $FLAGS -x hip -I"$R/blt_amd/csrc" -c "${HSRC:-$R/blt_amd/csrc/blt_host.cpp}" -o "$R/build/exp/h_$NAME.o" &
$HIPCC $HF $FLAGS -x hip -c "$R/blt_amd/csrc/blt_pipeline.cpp" -o "$R/build/exp/p_$NAME.o" &
$HIPCC $HF $FLAGS ${KFLAGS:-} -I"$R/blt_amd/csrc" -c "${KSRC:-$R/blt_amd/csrc/bpe_kernels.hip}" -o "$R/build/exp/k_$NAME.o"
wait
mkdir -p "$R/build/xp"; $HIPCC $HF -shared -o "$R/build/xp/libblt_bpe_$NAME.so" "$R/build/exp/k_$NAME.o" "$R/build/exp/h_$NAME.o" "$R/build/exp/p_$NAME.o" -lpthread
echo "built build/xp/libblt_bpe_$NAME.so ($FLAGS)"
