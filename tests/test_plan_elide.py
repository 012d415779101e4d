"""Step-plan link elision (kdfm/plan.py _elide_links) on synthetic op lists: a record repeating the previous one
at the same point of its stream is dropped with the waits that already bound to that point; main-stream work in
between, a launch naming none of the linked streams, a host callback, or a new waiter keep the link."""
import ctypes as C

from kdfm import plan

M, S, T = 0x7f0000001000, 0x7f0000002000, 0x7f0000003000


def _fn(name):
    f = lambda *a: 0  # noqa: E731
    f.__name__ = name
    return f


REC, WAIT, KER, OTHER = _fn("kdfm_event_record"), _fn("kdfm_stream_wait_event"), _fn("kdfm_ffn_bwd"), _fn("kdfm_set")


def k(fn, *args):
    return ("k", fn, args, 0)


def names(ops):
    return [(o[1].__name__ if o[0] == "k" else o[0], o[2]) for o in ops]


def test_repeated_fork_is_elided():
    ops = [k(KER, 1, M), k(REC, 7, M), k(WAIT, S, 7), k(KER, 2, S),
           k(REC, 7, M), k(WAIT, S, 7), k(KER, 3, S)]
    out = plan._elide_links(ops)
    assert names(out) == names(ops[:4] + ops[6:])


def test_main_stream_work_between_keeps_the_link():
    ops = [k(REC, 7, M), k(WAIT, S, 7), k(KER, 2, S), k(KER, 1, M), k(REC, 7, M), k(WAIT, S, 7)]
    assert len(plan._elide_links(ops)) == len(ops)


def test_wait_on_the_recording_stream_between_keeps_the_link():
    ops = [k(REC, 7, M), k(WAIT, S, 7), k(REC, 8, T), k(WAIT, M, 8), k(REC, 7, M), k(WAIT, S, 7)]
    assert len(plan._elide_links(ops)) == len(ops)


def test_unattributed_launch_and_host_callback_are_barriers():
    ops = [k(REC, 7, M), k(WAIT, S, 7), k(OTHER, 5, 6), k(REC, 7, M), k(WAIT, S, 7)]
    assert len(plan._elide_links(ops)) == len(ops)
    ops = [k(REC, 7, M), k(WAIT, S, 7), ("py", print, ()), k(REC, 7, M), k(WAIT, S, 7)]
    assert len(plan._elide_links(ops)) == len(ops)


def test_new_waiter_keeps_its_wait():
    ops = [k(REC, 7, M), k(WAIT, S, 7), k(REC, 7, M), k(WAIT, S, 7), k(WAIT, T, 7)]
    out = plan._elide_links(ops)
    assert names(out) == names([ops[0], ops[1], ops[4]])


def test_torch_event_ops():
    ev, m, s = C.c_void_p(7), C.c_void_p(M), C.c_void_p(S)
    ops = [("er", ev, m), ("ew", ev, s), k(KER, 2, S), ("er", ev, m), ("ew", ev, s)]
    assert len(plan._elide_links(ops)) == 3
