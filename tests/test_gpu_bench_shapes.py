"""Parity of the exact shapes bench.py times (VERDICT r5 ask 3): the headline's four
batches in flight (256 k=128 squares each, CEL_FLAG_CALLER_STREAM on four streams,
bench.py --inflight 4), the k=512 rider (four batches of 32 GF(2^16) squares) and the
config-4 k=64 rider (four batches of 1024 squares). The batches are built and stepped the
way bench._measure_batch does it (SquareBatch per batch, ODS placed in Q0, the distinct
synthetic squares rotated by one per batch, steps dealt round robin), then every square's
DAH and 4k roots and every status are checked against the oracle
(pkg/da/data_availability_header.go:44-75), and sampled squares' EDS bytes (the whole
EDS at k <= 128, a digest at k = 512)."""
import hashlib

import numpy as np
import pytest

from celestia_eds.testfactory import random_ods

pytestmark = pytest.mark.gpu


def _run_inflight(oracle, k, B, inflight, n_distinct, steps, eds_samples, seed):
    import torch
    from celestia_eds.device import SquareBatch

    distinct = [random_ods(k, seed + i) for i in range(n_distinct)]
    expect = [oracle.extend_and_commit(d) for d in distinct]
    sbs = []
    for j in range(inflight):
        sb = SquareBatch(B, k, ods_in_eds=True)
        sb.load_ods(torch.from_numpy(np.stack([distinct[(i + j) % n_distinct] for i in range(B)])))
        sb.status.fill_(0x7F7F7F7F)
        sbs.append(sb)
    torch.cuda.synchronize()
    for i in range(steps):  # as bench.py: steps dealt to the batches in turn
        sbs[i % inflight].extend_and_commit(caller_stream=True)
    torch.cuda.synchronize()
    w = 2 * k
    for j, sb in enumerate(sbs):
        st = sb.status.cpu().numpy()
        assert (st == 0).all(), f"batch {j}: status {st[st != 0][:4]}"
        dah = sb.dah.cpu().numpy()
        rr, cr = sb.row_roots.cpu().numpy(), sb.col_roots.cpu().numpy()
        for i in range(B):
            e = expect[(i + j) % n_distinct]
            assert dah[i].tobytes() == e[3], f"batch {j} square {i}: DAH differs"
            assert np.array_equal(rr[i], e[1]) and np.array_equal(cr[i], e[2]), f"batch {j} square {i}: roots differ"
        for sq in eds_samples:
            eds = sb.eds[sq].cpu().numpy()
            want = expect[(sq + j) % n_distinct][0]
            assert eds.shape == (w, w, 512)
            if k >= 512:
                assert hashlib.sha256(eds.tobytes()).digest() == hashlib.sha256(want.tobytes()).digest(), \
                    f"batch {j} square {sq}: EDS digest differs"
            else:
                assert np.array_equal(eds, want), f"batch {j} square {sq}: EDS differs"
    del sbs
    torch.cuda.empty_cache()


def test_headline_four_batches_in_flight(oracle):
    """bench.py default line: k=128, 256 squares per batch, --inflight 4, 4 distinct
    squares, 8 steps (every batch stepped twice, the second step of each batch waiting on
    the previous batch's extension event)."""
    _run_inflight(oracle, 128, 256, 4, 4, 8, (0, 131, 255), 9300)


def test_k512_rider_four_batches(oracle):
    """The k512 rider: 4 batches of 32 k=512 squares in flight, 2 distinct squares."""
    _run_inflight(oracle, 512, 32, 4, 2, 6, (0, 31), 9400)


def test_k64_rider_four_batches(oracle):
    """The config-4 rider at N = 1: 1024 k=64 squares per batch, 4 batches in flight,
    4 distinct squares (the N = 8 share, 128 squares per batch, is the k64 batch tests)."""
    _run_inflight(oracle, 64, 1024, 4, 4, 6, (0, 513, 1023), 9500)
