#!/bin/bash
# tools/ab_build.sh NAME [hipcc flags...] -- build an A/B variant of the loop
# kernel from the working tree: qpsk-modulator-demodulator_amd/_build/ab/libNAME.so
# (the library with qpsk_loop.o rebuilt under the extra flags, every other
# object from the in-tree build) and tools/bin/loop_probe_NAME (the stamped
# diagnostic build).  Run `make -C qpsk-modulator-demodulator_amd` first.
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/qpsk-modulator-demodulator_amd
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I$root/include -I$pkg/csrc -mllvm -amdgpu-sched-strategy=max-ilp"
mkdir -p "$pkg/_build/ab" "$root/tools/bin"
/opt/rocm/bin/hipcc $flags "$@" -c "$pkg/csrc/qpsk_loop.hip" -o "$pkg/_build/ab/loop_$name.o" 2> /dev/null
objs=$(ls "$pkg"/_build/*.o | grep -v '/qpsk_loop.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$pkg/_build/ab/lib$name.so" $objs "$pkg/_build/ab/loop_$name.o"
/opt/rocm/bin/hipcc $flags "$@" "$root/tools/loop_probe.hip" -o "$root/tools/bin/loop_probe_$name" 2> /dev/null
echo "built lib$name.so loop_probe_$name"
