"""The library's ReSTIR DI halo exchange plan (mpt_halo_plan, the operations mpt_set_halo_native's
RCCL exchange issues): host logic, no GPU.

* Every band's receives are exactly mpt.partition.halo_plan's (the Python exchange the bench's
  torch.distributed path runs and the gloo / in-process tests pin bit-exact), and so are its sends.
* The point-to-point operations pair up: for every pair of bands (k, p), the sends k issues to p
  and the receives p issues from k are the same buffers and rows in the same order -- what
  ncclSend / ncclRecv need inside one group, or every rank hangs.
* Bytes: what a band receives is what its peers send it (the one-GPU rehearsal, mode 2, moves the
  receive total; tests/test_halo_native.py checks that figure on the GPU).
"""
import itertools

import pytest

from mpt import partition

# (res_y, bands, halo rows): the 8-way 1080p split at the C4 halos, bands smaller than the halo
# (a receive from two peers), a ragged split with an empty last band, halo 0
CASES = [(1080, 8, h) for h in (0, 3, 28, 135, 136, 300)] + \
        [(1080, 4, 28), (1080, 2, 700), (96, 4, 28), (64, 3, 5), (9, 4, 2), (9, 4, 7), (27, 5, 4), (1, 1, 3)]


def _plan(res_y, nb, h, k, n_buffers):
    import mpt
    bh = partition.contiguous_band(res_y, nb, 0)[0]
    return bh, mpt.halo_plan(res_y, bh, nb, k, h, n_buffers)


@pytest.mark.parametrize("res_y,nb,h", CASES)
def test_halo_plan_matches_partition_plan(res_y, nb, h):
    for k in range(nb):
        bh, ops = _plan(res_y, nb, h, k, 1)
        sends, recvs = partition.halo_plan(res_y, bh, nb, k, h)
        got_s = sorted((p, lo, hi) for (p, kind, _, lo, hi) in ops if kind == "send")
        got_r = sorted((p, lo, hi) for (p, kind, _, lo, hi) in ops if kind == "recv")
        assert got_s == sends, (k, got_s, sends)
        assert got_r == recvs, (k, got_r, recvs)


@pytest.mark.parametrize("res_y,nb,h", CASES)
@pytest.mark.parametrize("n_buffers", [1, 5, 12])
def test_halo_plan_sends_and_receives_pair_up(res_y, nb, h, n_buffers):
    plans = {k: _plan(res_y, nb, h, k, n_buffers)[1] for k in range(nb)}
    for k, p in itertools.permutations(range(nb), 2):
        sent = [(b, lo, hi) for (q, kind, b, lo, hi) in plans[k] if q == p and kind == "send"]
        got = [(b, lo, hi) for (q, kind, b, lo, hi) in plans[p] if q == k and kind == "recv"]
        assert sent == got, (k, p, sent, got)
    for k in range(nb):
        ops = plans[k]
        peers = [q for (q, *_rest) in ops]
        assert peers == sorted(peers) and k not in peers      # peer order, never itself
        for (q, kind, b, lo, hi) in ops:
            assert 0 <= b < n_buffers and 0 <= lo < hi <= res_y
            bh = partition.contiguous_band(res_y, nb, 0)[0]
            own = (min(res_y, k * bh), min(res_y, k * bh + bh))
            rows = (lo, hi)
            if kind == "send":     # a band only ever sends its own rows ...
                assert own[0] <= rows[0] and rows[1] <= own[1]
            else:                  # ... and receives rows of its halo from their owner
                assert rows[1] <= own[0] or rows[0] >= own[1]
                assert min(res_y, q * bh) <= lo and hi <= min(res_y, q * bh + bh)
                assert lo >= own[0] - h and hi <= own[1] + h


def test_halo_plan_8way_1080p_bytes():
    """The C4 8-way split's receive volume at the default reuse halo: every interior band takes
    2 x halo rows per buffer, the edge bands one side."""
    res_y, nb, h = 1080, 8, 28
    for k in range(nb):
        _, ops = _plan(res_y, nb, h, k, 3)
        rows = sum(hi - lo for (_, kind, _, lo, hi) in ops if kind == "recv")
        assert rows == 3 * h * (1 if k in (0, nb - 1) else 2)


def test_halo_plan_rejects_bad_arguments():
    import mpt
    with pytest.raises(mpt.MptError):
        mpt.halo_plan(1080, 135, 8, 8, 28)
    with pytest.raises(mpt.MptError):
        mpt.halo_plan(1080, 135, 8, 0, -1)
    with pytest.raises(mpt.MptError):
        mpt.halo_plan(1080, 135, 8, 0, 28, 13)
