#!/bin/bash
# Build an experimental variant of libseriation.so with extra device defines:
#   tools/build_variant.sh NAME "-DSR_STAMPS"  ->  <pkg>/build/var/NAME/libseriation.so
#   SRC=path/to/sr_device.hip tools/build_variant.sh NAME ""   (another version of the kernel source)
set -e
cd "$(dirname "$0")/../seriation-in-paleontological-data-using-mcmc_amd"
make -s build/sr_host.o build/sr_post.o
D=build/var/$1
mkdir -p "$D"
SRCF=${SRC:-csrc/sr_device.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function \
  -I../include -Icsrc $2 -c -o "$D/sr_device.o" -x hip "$SRCF"
/opt/rocm/bin/hipcc -shared -fPIC -o "$D/libseriation.so" build/sr_host.o "$D/sr_device.o" build/sr_post.o -lm -pthread
echo "$D/libseriation.so"
