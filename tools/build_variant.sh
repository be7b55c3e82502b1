#!/bin/bash
# Build an experiment variant of libdnrp.so: tools/build_variant.sh NAME "FLAGS" src1 [src2 ...]
# recompiles the listed sources (paths under dect-nr-plus-sdr_amd/csrc) with FLAGS and links
# dect-nr-plus-sdr_amd/libdnrp_NAME.so from them and the regular objects; select it with DNRP_LIB.
set -e
name=$1; flags=$2; shift 2
cd "$(dirname "$0")/../dect-nr-plus-sdr_amd"
make -s
out=build/variant_$name
mkdir -p $out
objs=""
for o in $(find build/host build/kernels -name "*.o" | sort); do objs="$objs $o"; done
for src in "$@"; do
  base=$(basename $src)
  sub=$(basename $(dirname $src))
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags \
      -I../include -Icsrc/host -Icsrc/kernels -Ibuild/gen $( case "$base" in tx.hip|rx.hip|rx_back.hip|rx_fused.hip|rx_epoch.hip) echo -fno-slp-vectorize ;; esac ) \
      -c csrc/$sub/$base -o $out/$base.o
  objs=$(echo $objs | tr ' ' '\n' | grep -v "build/$sub/$base.o" | tr '\n' ' ')
  objs="$objs $out/$base.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o libdnrp_$name.so $objs
echo "built dect-nr-plus-sdr_amd/libdnrp_$name.so"
