#!/bin/bash
# tools/ab_build_fll.sh NAME [SRC] [hipcc flags...] -- an A/B variant of the FLL:
# qpsk-modulator-demodulator_amd/_build/ab/libNAME.so = the in-tree library with
# qpsk_fll.o rebuilt from SRC (default csrc/qpsk_fll.hip) under the extra flags
# (e.g. -DNAME=VALUE for an A/B macro).  Run `make -C qpsk-modulator-demodulator_amd` first.
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/qpsk-modulator-demodulator_amd
src=$pkg/csrc/qpsk_fll.hip
if [ $# -gt 0 ] && [ -f "$1" ]; then src=$(cd "$(dirname "$1")" && pwd)/$(basename "$1"); shift; fi
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -I$root/include -I$pkg/csrc -mllvm -misched=ilpmin"
mkdir -p "$pkg/_build/ab"
/opt/rocm/bin/hipcc $flags "$@" -c "$src" -o "$pkg/_build/ab/fll_$name.o" 2> /dev/null
objs=$(ls "$pkg"/_build/*.o | grep -v '/qpsk_fll.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$pkg/_build/ab/lib$name.so" $objs "$pkg/_build/ab/fll_$name.o"
echo "built lib$name.so"
