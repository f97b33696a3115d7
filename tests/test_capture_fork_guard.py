"""CPU: the capture_fork guard (update.capture_fork_check) against the fork / join patterns of
tools/capture_fork_probe.py -- it must reject exactly the ones that segfaulted hipStreamEndCapture on the
GPU (profiles/r05_capture_fork_probe.txt) and accept the ones that captured, and the product's own
pipelined schedule must pass it."""
import pytest

from foundationstereo_amd import update as up


class S:                                   # a stream stand-in: identity only (or a HIP handle)
    def __init__(self, name, handle=None):
        self.name = name
        if handle is not None:
            self.cuda_stream = handle


def run(pattern):
    """Replay a probe variant's waits ((waiter, waited) pairs; 'cur' = the capture origin)."""
    cur, A, X = S("cur"), S("A"), S("X")
    names = {"cur": cur, "A": A, "X": X}
    side = {up._skey(A), up._skey(X)}
    up.capture_fork_check(cur, cur, capturing=False)          # a new capture: no edges
    for w, d in pattern:
        up.capture_fork_check(names[w], names[d], capturing=True, side_ids=side)


# the probe's variants as waits (waiter, waited), in issue order (tools/capture_fork_probe.py)
VARIANTS = {
    "a_only": [("A", "cur"), ("X", "A"), ("A", "X"), ("cur", "A")],
    "main_only": [("X", "cur"), ("cur", "X"), ("X", "cur"), ("cur", "X")],
    "two_parents": [("X", "cur"), ("cur", "X"), ("A", "cur"), ("X", "A"), ("A", "X"), ("cur", "A")],
    "two_parents_mainjoin": [("X", "cur"), ("cur", "X"), ("A", "cur"), ("X", "A"), ("A", "X"), ("cur", "A"),
                             ("cur", "X")],
    "via_main": [("A", "cur"), ("X", "cur"), ("A", "X"), ("cur", "A"), ("cur", "X")],
    "via_main_nojoin": [("A", "cur"), ("X", "cur"), ("A", "X"), ("cur", "A")],
    "enter_main_wait_side": [("X", "cur"), ("A", "cur"), ("X", "A"), ("A", "X"), ("cur", "A"), ("cur", "X")],
    "reenter_main_wait_side": [("X", "cur"), ("cur", "X"), ("X", "cur"), ("A", "cur"), ("X", "A"), ("A", "X"),
                               ("cur", "A"), ("cur", "X")],
}
SEGFAULTED = {"a_only", "two_parents", "two_parents_mainjoin", "enter_main_wait_side", "reenter_main_wait_side"}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_guard_matches_probe(name):
    if name in SEGFAULTED:
        with pytest.raises(up.CaptureForkError):
            run(VARIANTS[name])
    else:
        run(VARIANTS[name])


def test_not_capturing_records_nothing():
    A, X = S("A"), S("X")
    side = {up._skey(A), up._skey(X)}
    up.capture_fork_check(A, X, capturing=False, side_ids=side)
    up.capture_fork_check(X, A, capturing=False, side_ids=side)
    up.capture_fork_check(A, X, capturing=True, side_ids=side)   # fresh capture: fine


def test_streams_identified_by_handle():
    """torch.cuda.current_stream() hands out a fresh wrapper per call: two wrappers of one HIP stream are
    the same stream to the guard (round 6: the guard keyed on id() and missed the real pipeline fork)."""
    A1, A2, X = S("A", handle=0x1000), S("A", handle=0x1000), S("X", handle=0x2000)
    side = {up._skey(A1), up._skey(X)}
    up.capture_fork_check(A1, X, capturing=False, side_ids=side)
    up.capture_fork_check(X, A1, capturing=True, side_ids=side)      # X waits on A
    with pytest.raises(up.CaptureForkError):
        up.capture_fork_check(A2, X, capturing=True, side_ids=side)  # A (another wrapper) waits on X
