cd /root/repo
export TMPDIR=/tmp
VTAG=_32 bash tools/bench_variants.sh && VTAG=_64 bash tools/bench_variants.sh --workload sharded
