"""Self-describing byte comparisons for the host-path tests (VERDICT r4 item 1:
a failure must name its bytes).  On a mismatch the message gives, per array
that differs: how many bytes differ, the first and last differing offset, the
array's address modulo 4096 (the page placement of the caller's memory)."""
import numpy as np


def _addr(a):
    try:
        return int(np.asarray(a).ctypes.data)
    except Exception:  # noqa: BLE001 -- views without a data pointer
        return -1


def describe(got, want, name="array"):
    """None when got equals want, else a one-line description of the difference."""
    g, w = np.asarray(got).reshape(-1), np.asarray(want).reshape(-1)
    if g.shape != w.shape:
        return f"{name}: shape {g.shape} != {w.shape}"
    bad = np.flatnonzero(g != w)
    if len(bad) == 0:
        return None
    a = _addr(got)
    return (f"{name}: {len(bad)} byte(s) differ, first at {int(bad[0])}, last at {int(bad[-1])} "
            f"(of {len(g)}; address % 4096 = {a % 4096 if a >= 0 else '?'})")


def assert_same(got_list, want_list, what=""):
    """Assert every array of got_list equals its counterpart, naming each that differs."""
    msgs = []
    for i, (g, w) in enumerate(zip(got_list, want_list)):
        d = describe(g, w, f"[{i}]")
        if d:
            msgs.append(d)
    assert not msgs, f"{what}: " + "; ".join(msgs)
