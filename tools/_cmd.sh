cd /root/repo
export TMPDIR=/tmp
VTAG=_32 bash tools/bench_variants.sh && VTAG=_32b bash tools/bench_variants.sh
