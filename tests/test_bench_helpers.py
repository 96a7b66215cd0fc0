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
