#!/bin/bash
# Build a variant of libkarma_hip.so with extra compile flags (e.g. -DKARMA_CLS_WAVES=6)
# into karma_amd/variants/libkarma_<name>.so; select it with KARMA_LIB=... at run time.
# Usage: tools/build_variant.sh NAME "-DFOO=1 -DBAR=2"   (SRC=dir: sources other than karma_amd/csrc,
# e.g. a `git archive` of an earlier commit, for before/after timing)
set -e
NAME=$1; shift
EXTRA="$*"
REPO=$(cd "$(dirname "$0")/.." && pwd)
SRC=${SRC:-$REPO/karma_amd/csrc}
OUT=$REPO/karma_amd/variants
B=$OUT/build_$NAME
mkdir -p $B
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result -Wno-unused-value"
HASH=$(cat $(ls $SRC/*.hip $SRC/*.h $SRC/*.cpp $REPO/include/karma.h | sort) | sha256sum | cut -c1-16)
# the variant's -D flags are recorded in karma_build_info() (bench.py refuses
# a variant unless KARMA_ALLOW_VARIANT=1)
/opt/rocm/bin/hipcc $FLAGS $EXTRA -DKARMA_BUILD_DEFINES="\"$EXTRA\"" -DKARMA_SRC_HASH="\"$HASH\"" -c $SRC/core.hip -o $B/core.o &
pids="$!"
for f in kmer graph graph_sets eq consumers comm step sort; do
  /opt/rocm/bin/hipcc $FLAGS $EXTRA -c $SRC/$f.hip -o $B/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fopenmp -x c++ -c $SRC/synth.cpp -o $B/synth.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -pthread -x c++ -c $SRC/ingest.cpp -o $B/ingest.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fopenmp -o $OUT/libkarma_$NAME.so $B/*.o -L/opt/rocm/lib/llvm/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $B
echo built $OUT/libkarma_$NAME.so
