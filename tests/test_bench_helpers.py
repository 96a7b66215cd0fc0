"""bench.py's line helpers on CPU: the chain-protocol record decodes
gnoc_summary.chain_protocol as include/gnoc.h documents it (bit 8 chain engine,
bits 0 / 1 look-back per phase, bit 10 the M/G/1
instantiation, bit 11 only its windows on it)."""
import bench


def test_chain_protocol_bits():
    assert bench.chain_protocol({"chain_protocol": 0}) is None
    assert bench.chain_protocol({"chain_protocol": 0x100}) == {"x": "serial", "y": "serial",
                                                              "mg1_serial": False, "mg1_split": False}
    got = bench.chain_protocol({"chain_protocol": 0x100 | 2 | 0x400 | 0x800})
    assert got == {"x": "serial", "y": "lookback", "mg1_serial": True, "mg1_split": True}
    got = bench.chain_protocol({"chain_protocol": 0x100 | 1})
    assert got["x"] == "lookback" and not got["mg1_serial"]


class _FakeEngine:
    """Counts runs; its windows change on the first `adapt` runs (variable windows)."""

    def __init__(self, adapt):
        self.adapt, self.runs, self.prof, self.timed_prof = adapt, 0, False, 0

    def run(self):
        self.runs += 1
        if self.prof:
            self.timed_prof += 1

    def summary(self):
        w = 100 + min(self.runs, self.adapt)
        return {"windows": w, "windows_y": w, "window_ps_x": 1, "window_ps_y": 1, "retries": 0, "fallbacks": 0,
                "retries_total": 0, "fallbacks_total": 0, "runs": self.runs}

    def set_profiling(self, on):
        self.prof = on

    def kernel_stats(self):
        return {}


class _Args:
    steps, warmup = 5, 1


def test_measure_settles_before_timing():
    """At least SETTLE_MIN runs before the warmup, more while the windows still change,
    then exactly `steps` timed runs and one profiled run."""
    for adapt, fixed in ((0, False), (3, False), (20, False), (20, True)):
        eng = _FakeEngine(adapt)
        m = bench.measure(eng, _Args, lambda: None, settle_fixed=fixed)
        settle = m["settle_runs"]
        assert settle >= bench.SETTLE_MIN
        if fixed:
            assert settle == bench.SETTLE_MIN
        elif adapt < bench.SETTLE_MIN:
            assert settle == bench.SETTLE_MIN
        else:
            assert settle == adapt + 1
        assert m["reruns"]["timed_runs"] == _Args.steps
        assert eng.runs == settle + _Args.warmup + _Args.steps + 1 and eng.timed_prof == 1
