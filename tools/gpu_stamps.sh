#!/bin/bash
# Chain stamps of the current sources (libgnoc_stamps.so, a -DCH_STAMPS build): uniform and hotspot.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so CH_STAMPS_DUMP=gpurun_out/${TAG}_st timeout -k 10 200 python3 -u tools/chain_stamps.py > gpurun_out/${TAG}_stamps.txt 2>&1 &&
GNOC_LIB=graphite_amd/_build/libgnoc_stamps.so timeout -k 10 200 python3 -u tools/chain_stamps.py 32 0.005 10000 hotspot > gpurun_out/${TAG}_stamps_hot.txt 2>&1
rc=$?
cat gpurun_out/${TAG}_stamps.txt
exit $rc
