#!/bin/bash
# Build an experimental variant of libseriation.so with extra device defines:
#   tools/build_variant.sh NAME "-DSR_STAMPS"  ->  <pkg>/build/var/NAME/libseriation.so
#   SRC=path/to/sr_device.hip tools/build_variant.sh NAME ""   (another version of the kernel source)
# The variant is self-contained: its own source snapshot (build/var/NAME/spec/, the variant's kernel
# source) and hash, and the same extra defines for its shape-specialised kernels (SR_SPEC_EXTRA), so a
# session of the variant runs the variant's specialised kernel, like the product library does.
set -e
cd "$(dirname "$0")/../seriation-in-paleontological-data-using-mcmc_amd"
make -s build/sr_host.o build/sr_post.o build/srhash
D=build/var/$1
mkdir -p "$D/spec"
SRCF=${SRC:-csrc/sr_device.hip}
cp csrc/sr_math.h csrc/sr_rng.h csrc/sr_tables.h csrc/sr_internal.h ../include/seriation.h "$D/spec/"
cp "$SRCF" "$D/spec/sr_device.hip"
H=$(build/srhash "$D/spec")
gcc -O2 -std=gnu11 -pthread -fPIC -ffp-contract=off -fno-fast-math -Wall -I../include -Icsrc \
  -DSR_SPEC_HASH=0x${H}ull -DSR_ARCH='"gfx950"' -DSR_SPEC_EXTRA="\"$2\"" -c -o "$D/sr_spec.o" csrc/sr_spec.c
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -mllvm -disable-machine-licm -Wall -Wno-unused-function \
  -I../include -Icsrc $2 -c -o "$D/sr_device.o" -x hip "$SRCF"
/opt/rocm/bin/hipcc -shared -fPIC -o "$D/libseriation.so" build/sr_host.o "$D/sr_device.o" build/sr_post.o "$D/sr_spec.o" -ldl -lm -pthread
echo "$D/libseriation.so"
# its specialised kernels for the reference's datasets and the bench matrix, compiled now (a profiled run of
# the variant finds them instead of falling back to its generic kernel: no compile under a profiler)
(cd .. && SERIATION_LIB="$PWD/seriation-in-paleontological-data-using-mcmc_amd/$D/libseriation.so" python3 -c \
  "import __graft_entry__ as g; print('prewarm', g.prewarm(test_shapes=False))")
