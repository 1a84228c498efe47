"""GPU tests: one codec handle shared by several host threads, each enqueueing
the device-batch calls on its own stream (the handle is
immutable after create and safe for concurrent calls, like the reference's
static final codec).  The first calls race to build the cached decode plans,
their device images and the pattern tables; every thread's bytes must still
be exact.
"""
import itertools
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED


def test_shared_codec_many_streams(gpu, oracle_lib):
    import torch
    import rsamd
    from rsamd import device
    from rsamd.device import StripeLayout
    k, m, S, B = 4, 2, 64 << 10, 64
    rs = rsamd.ReedSolomon.create(k, m)  # fresh: no plan cached yet
    pats = [tuple(i not in miss for i in range(6))
            for e in (1, 2) for miss in itertools.combinations(range(6), e)]
    errors = []
    barrier = threading.Barrier(6)

    def work(w):
        try:
            torch.cuda.set_device(0)
            st = torch.cuda.Stream()
            lay = StripeLayout.packed(B, k + m, S)
            with torch.cuda.stream(st):
                buf = torch.empty(lay.nbytes, dtype=torch.uint8, device="cuda:0")
                flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")
            device.fill_synthetic(buf.data_ptr(), k, lay, SEED, 1000 * w, st)
            v = buf.view(B, k + m, S)
            barrier.wait()
            device.encode(rs, buf.data_ptr(), lay, st)
            device.verify(rs, buf.data_ptr(), lay, flag.data_ptr(), st)
            st.synchronize()
            assert int(flag.item()) == 0
            good = v.clone()
            for present in pats[w::6]:  # each thread its own erasure patterns
                miss = [i for i in range(6) if not present[i]]
                with torch.cuda.stream(st):
                    v[:, miss, :] = 0x33
                device.decode(rs, buf.data_ptr(), list(present), lay, st)
                st.synchronize()
                assert torch.equal(v, good), (w, miss)
            # per-stripe patterns through the host-flag call (pattern tables)
            present = np.array([pats[(w + t) % len(pats)] for t in range(B)], dtype=bool)
            with torch.cuda.stream(st):
                v[torch.from_numpy(~present).to("cuda:0")] = 0x77
            device.decode_masked(rs, buf.data_ptr(), present, lay, st)
            st.synchronize()
            assert torch.equal(v, good), w
            first = good[0].cpu().numpy()
            ref = [x.copy() for x in first]
            ref[4][:] = 0
            ref[5][:] = 0
            oracle_lib.Codec(k, m).encode_parity(ref, 0, S)
            assert all(np.array_equal(a, b) for a, b in zip(first, ref)), w
        except Exception as e:  # noqa: BLE001
            errors.append((w, repr(e)))

    ts = [threading.Thread(target=work, args=(w,)) for w in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


def test_thread_exit_releases_its_staging(gpu, oracle_lib):
    """A worker thread's host-API contexts (streams, device staging, pinned
    mirrors) are freed when the thread exits (JVM / gRPC pools retire
    threads), not leaked until rs_thread_release."""
    import torch
    import rsamd
    torch.cuda.synchronize()
    n = 48 << 20
    rng = np.random.default_rng(1)
    sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8) for _ in range(2)]
    ref = [a.copy() for a in sh]
    oracle_lib.Codec(4, 2).encode_parity(ref, 0, n)
    rs = rsamd.ReedSolomon.create(4, 2)
    seen = {}

    def work():
        rs.encodeParity(sh, 0, n)
        seen["mid"] = torch.cuda.mem_get_info()[0]

    free0 = torch.cuda.mem_get_info()[0]
    t = threading.Thread(target=work)
    t.start()
    t.join()
    assert all(np.array_equal(a, b) for a, b in zip(sh, ref))
    held = free0 - seen["mid"]
    if held > (32 << 20):  # the thread held staging memory while it lived
        # join() returns before the pthread has run its thread-local destructors: poll
        import time
        t0 = time.time()
        while True:
            free1 = torch.cuda.mem_get_info()[0]
            if free1 - seen["mid"] >= 0.8 * held or time.time() - t0 > 5:
                break
            time.sleep(0.05)
        assert free1 - seen["mid"] >= 0.8 * held, (free0, seen["mid"], free1)


def test_retired_contexts_are_reused(gpu, oracle_lib):
    """Workers that come and go (a JVM / gRPC pool): each exiting thread's
    contexts go to the reaper, which frees their buffers and keeps their
    streams for the next new thread (host.cpp orphan / adopt_idle).  Six
    short-lived workers in turn, alternating calls on the direct path (6 MiB
    per shard, page-locked for the call) and on the zero-copy staging buffer
    (40 KB), all bit-exact."""
    import rsamd
    rs = rsamd.ReedSolomon.create(4, 2)
    oc = oracle_lib.Codec(4, 2)
    errors = []

    def work(seed, n):
        try:
            rng = np.random.default_rng(seed)
            sh = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(4)] + [np.zeros(n, np.uint8)
                                                                                 for _ in range(2)]
            ref = [a.copy() for a in sh]
            oc.encode_parity(ref, 0, n)
            rs.encodeParity(sh, 0, n)
            assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), seed
            sh[1][:] = 0
            sh[5][:] = 0
            rs.decodeMissing(sh, [True, False, True, True, True, False], 0, n)
            assert all(np.array_equal(a, b) for a, b in zip(sh, ref)), seed
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    for seed in range(6):
        t = threading.Thread(target=work, args=(seed, (6 << 20) + seed if seed % 2 else 40_000 + seed))
        t.start()
        t.join()
    assert not errors, errors
