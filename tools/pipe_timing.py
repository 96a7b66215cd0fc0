"""Per-port cycle breakdown of the port pipelines (a -DPIPE_TIMING build):
    GNOC_LIB=graphite_amd/_build/libgnoc_timing.so python tools/pipe_timing.py LOG
reads the GNOC_PIPE_DEBUG_ALL records tools/pipe_dbg.py printed into LOG (the last run)."""
import re
import sys

lines = open(sys.argv[1]).read().split('\n')
runs = [i for i, l in enumerate(lines) if l.startswith('run ')]
blk = lines[runs[-2] + 1:runs[-1]] if len(runs) > 1 else lines
for ph in 'XY':
    ports, svcs = [], []
    for l in blk:
        m = re.match(r'gnoc pipe %s (port|svc) #(\d+) why (\d+): (.*)' % ph, l)
        if not m:
            continue
        a, b = m.group(4).split('|')
        st, tm = list(map(int, a.split())), list(map(int, b.split()))
        (ports if m.group(1) == 'port' else svcs).append((int(m.group(2)), st, tm))
    if not ports:
        continue
    K = lambda x: x * 256 / 1000
    ports.sort(key=lambda p: -p[2][6])
    print(f"{ph}: {len(ports)} ports; busiest (k cycles; per-row cycles in brackets)")
    for k, st, tm in ports[:6]:
        rows = max(1, st[14])
        parts = " ".join(f"{nm} {K(tm[q]):.0f} [{tm[q] * 256 / rows:.0f}]" for nm, q in
                         (("cand+merge", 7), ("rowrd", 8), ("scan", 9), ("out", 10)))
        print(f"  #{k} i={st[0]} n={tm[6]} rows={st[14]} short={tm[5]} total {K(tm[0]):.0f} wait_in {K(tm[1]):.0f} "
              f"wait_room {K(tm[2]):.0f} ymerge {K(tm[3]):.0f} row {K(tm[4]):.0f} | {parts}")
    svcs.sort(key=lambda p: -p[2][0])
    for k, st, tm in svcs[:3]:
        print(f"  svc #{k} c={st[0]} s={st[1]} total {K(tm[0]):.0f} rounds {tm[1]} idle {tm[2]} loads {tm[3]} links {tm[4]}")
