#!/bin/bash
# A/B timing of libgnoc variants on configs[1]: tools/gpu_ab.sh OUT v1 v2 ... , each run twice,
# interleaved.  A variant is "cur" (libgnoc.so), a suffix NAME (libgnoc_NAME.so), or either
# followed by "+VAR=VAL" settings for the run (e.g. cur+GNOC_CH_XCD=0); AB_HOT: hotspot fraction.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/$1; shift
: > $out
for rep in 1 2; do
  for v in "$@"; do
    name=${v%%+*}; envs=""; [ "$name" != "$v" ] && envs=${v#*+}
    lib=graphite_amd/_build/libgnoc.so; [ "$name" != cur ] && lib=graphite_amd/_build/libgnoc_$name.so
    echo "variant $v" >> $out
    env ${envs//+/ } GNOC_LIB=$lib timeout -k 10 120 python -u tools/run_probe.py 10 ${AB_HOT:-0} >> $out 2>&1 || { tail -5 $out; exit 1; }
  done
done
grep "^lib\|^variant" $out
