#!/bin/bash
# Build a libsr variant: tools/build_variant.sh NAME [extra hipcc flags...]
# -> schwarzschild-raytracer_amd/lib/variants/libsr_NAME.so (A/B timing only).
# KERNEL=path overrides the geodesic kernel source (e.g. a file made with
# `git show REV:schwarzschild-raytracer_amd/csrc/kernels/geodesic.hip`; it
# must match this tree's device_scene.h). WAVES: the small instantiation's
# waves per SIMD (default 7, the Makefile's).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/schwarzschild-raytracer_amd
NAME=$1; shift
KSRC=${KERNEL:-$PKG/csrc/kernels/geodesic.hip}
OBJ=$PKG/build/variants/$NAME; OUT=$PKG/lib/variants
mkdir -p "$OBJ" "$OUT"
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$ROOT/include -I$PKG/csrc -I$PKG/csrc/kernels -fno-slp-vectorize -DSR_MIN_WAVES_PER_EU=${WAVES:-7}"
H=/opt/rocm/bin/hipcc
$H $FLAGS --offload-arch=gfx950 -fno-gpu-rdc "$@" -x hip -c "$KSRC" -o $OBJ/geodesic.o &
$H $FLAGS --offload-arch=gfx950 -fno-gpu-rdc -x hip -c $PKG/csrc/kernels/assemble.hip -o $OBJ/assemble.o &
$H $FLAGS "$@" -c $PKG/csrc/sr_api.cpp -o $OBJ/sr_api.o &
$H $FLAGS -c $PKG/csrc/host/scene.cpp -o $OBJ/scene.o &
$H $FLAGS -c $PKG/csrc/host/png.cpp -o $OBJ/png.o &
$H $FLAGS -c $PKG/csrc/host/partition.cpp -o $OBJ/partition.o &
wait
$H -shared --offload-arch=gfx950 -Wl,-Bsymbolic -o $OUT/libsr_$NAME.so $OBJ/geodesic.o $OBJ/assemble.o $OBJ/sr_api.o $OBJ/scene.o $OBJ/png.o $OBJ/partition.o -lz
$H $FLAGS --offload-arch=gfx950 "$@" -x hip --cuda-device-only -S "$KSRC" -o $OBJ/geodesic.s
echo "$NAME: $(grep -E '^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count)' $OBJ/geodesic.s | head -3 | tr -s ' ' | tr '\n' ' ')"
