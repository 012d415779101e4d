"""The happens-before checker of tools/race_check.py (used by tests/test_race_gpu.py on the real
multi-stream step) on synthetic traces: vector-clock ordering through events, host synchronisation,
allocator reuse with and without record_stream, pruning, and the header-derived read/write sets."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import race_check as rc  # noqa: E402

A, B, Cs = 1, 2, 3   # three streams


class Ev:
    pass


def _t():
    return rc.Tracer(roles={A: "main", B: "side", Cs: "comm"})


def test_unordered_write_read_conflicts():
    t = _t()
    t.access(0, 100, A, True, "w", "k1")
    t.access(50, 60, B, False, "r", "k2")
    assert len(t.conflicts) == 1
    # read/read never conflicts
    t2 = _t()
    t2.access(0, 100, A, False, "r1", "k")
    t2.access(0, 100, B, False, "r2", "k")
    assert not t2.conflicts


def test_event_orders_streams():
    t = _t()
    t.access(0, 100, A, True, "w", "k1")
    e = Ev()
    t.record(e, A)
    t.wait(e, B)
    t.access(0, 100, B, False, "r", "k2")
    assert not t.conflicts
    # work issued on A after the record is not covered by the wait
    t.access(0, 100, A, True, "w2", "k3")
    assert len(t.conflicts) == 1


def test_event_rerecord_binds_at_wait():
    """StreamLink reuses one event: a wait binds to the record made before it."""
    t = _t()
    e = Ev()
    t.access(0, 8, A, True, "w1", "k")
    t.record(e, A)
    t.wait(e, B)
    t.access(0, 8, A, True, "w2", "k")
    t.record(e, A)       # re-recorded after B's wait: B is NOT ordered after w2
    t.access(0, 8, B, False, "r", "k")
    assert [k[0] for k in t.conflicts] == ["w2"]


def test_transitive_and_host_sync():
    t = _t()
    t.access(0, 8, A, True, "w", "k")
    e1, e2 = Ev(), Ev()
    t.record(e1, A)
    t.wait(e1, B)
    t.record(e2, B)
    t.wait(e2, Cs)
    t.access(0, 8, Cs, False, "r", "k")     # A -> B -> C
    assert not t.conflicts
    t.access(16, 24, B, True, "w2", "k")
    t.sync_all()
    t.access(16, 24, A, False, "r2", "k")
    assert not t.conflicts


def test_reuse_without_record_stream_is_a_race():
    """memory freed by its allocation stream A while stream B still reads it, then handed to a new
    tensor on A: a race unless B recorded itself on the old tensor (record_stream)."""
    t = _t()
    t.alloc(0, 64, A)
    t.access(0, 64, A, True, "produce", "k")
    e = Ev()
    t.record(e, A)
    t.wait(e, B)
    t.access(0, 64, B, False, "side-read", "k")
    t.alloc(0, 64, A)                           # freed + reallocated on A
    t.access(0, 64, A, True, "new-owner", "k")
    assert [k[0] for k in t.conflicts] == ["side-read"]
    assert list(t.conflicts.values())[0][1][-1] is True   # flagged as memory reuse

    t = _t()
    t.alloc(0, 64, A)
    t.access(0, 64, A, True, "produce", "k")
    t.record(e, A)
    t.wait(e, B)
    t.access(0, 64, B, False, "side-read", "k")
    t.record_stream(0, B)
    t.alloc(0, 64, A)
    t.access(0, 64, A, True, "new-owner", "k")
    assert not t.conflicts


def test_pruning_keeps_pages_small_and_exact():
    t = _t()
    for i in range(200):
        t.access(0, 4096, A, True, f"w{i}", "k")
    assert len(t.pages[0]) == 1
    t.access(0, 4096, B, False, "late", "k")
    assert len(t.conflicts) == 1 and next(iter(t.conflicts))[0] == "w199"


def test_header_read_write_sets():
    h = rc.parse_header()
    assert dict(h["kdfm_ffn_bwd"])["dout"] == "r" and dict(h["kdfm_ffn_bwd"])["dh_h"] == "w"
    assert dict(h["kdfm_ln_fold"])["parts"] == "rr" and dict(h["kdfm_ln_fold"])["dgamma"] == "ww"
    assert dict(h["kdfm_wgrad_bf16"])["ws"] == "w" and dict(h["kdfm_wgrad_bf16"])["X"] == "r"
    from kdfm import _lib
    for name, (_, args) in _lib.SIGNATURES.items():
        assert name in h and len(h[name]) == len(args), name
