#!/bin/bash
# tools/ab_build_obj.sh UNIT NAME [hipcc flags...] -- an A/B variant of one
# translation unit (qpsk_kernels, qpsk_loop, qpsk_fll, ...):
# qpsk-modulator-demodulator_amd/_build/ab/libNAME.so = the in-tree library with
# UNIT.o rebuilt from csrc/UNIT.hip under the extra flags (-D... switches).
# Run `make -C qpsk-modulator-demodulator_amd` first.
set -e
unit=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/qpsk-modulator-demodulator_amd
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$root/include -I$pkg/csrc"
case $unit in
  qpsk_fll) flags="$flags -fno-slp-vectorize -mllvm -amdgpu-sched-strategy=iterative-ilp" ;;
  qpsk_loop) flags="$flags -mllvm -amdgpu-sched-strategy=max-ilp" ;;
esac
mkdir -p "$pkg/_build/ab"
/opt/rocm/bin/hipcc $flags "$@" -c "$pkg/csrc/$unit.hip" -o "$pkg/_build/ab/${unit}_$name.o"
objs=$(ls "$pkg"/_build/*.o | grep -v "/$unit.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$pkg/_build/ab/lib$name.so" $objs "$pkg/_build/ab/${unit}_$name.o"
echo "built lib$name.so"
