#!/bin/bash
# Build a libsr variant: tools/build_variant.sh NAME [extra hipcc flags...]
# -> schwarzschild-raytracer_amd/lib/variants/libsr_NAME.so (A/B timing only)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/schwarzschild-raytracer_amd
NAME=$1; shift
OBJ=$PKG/build/variants/$NAME; OUT=$PKG/lib/variants
mkdir -p "$OBJ" "$OUT"
FLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$ROOT/include -I$PKG/csrc -fno-slp-vectorize -DSR_MIN_WAVES_PER_EU=6"
H=/opt/rocm/bin/hipcc
$H $FLAGS --offload-arch=gfx950 -fno-gpu-rdc "$@" -x hip -c $PKG/csrc/kernels/geodesic.hip -o $OBJ/geodesic.o &
$H $FLAGS "$@" -c $PKG/csrc/sr_api.cpp -o $OBJ/sr_api.o &
$H $FLAGS -c $PKG/csrc/host/scene.cpp -o $OBJ/scene.o &
$H $FLAGS -c $PKG/csrc/host/png.cpp -o $OBJ/png.o &
wait
$H -shared --offload-arch=gfx950 -Wl,-Bsymbolic -o $OUT/libsr_$NAME.so $OBJ/geodesic.o $OBJ/sr_api.o $OBJ/scene.o $OBJ/png.o -lz
$H $FLAGS --offload-arch=gfx950 "$@" -x hip --cuda-device-only -S $PKG/csrc/kernels/geodesic.hip -o $OBJ/geodesic.s
echo "$NAME: $(grep -E '^\s+\.(vgpr_count|sgpr_count|vgpr_spill_count)' $OBJ/geodesic.s | head -3 | tr -s ' ' | tr '\n' ' ')"
