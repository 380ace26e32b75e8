"""Storage-audit chunk selection (CPU) and chunk gather + hash (GPU) against the oracle's
restatement of c-pallets/audit/src/lib.rs:955-964 and numpy/hashlib."""
import hashlib

import numpy as np
import pytest

from cess_amd import audit


def test_need_count_matches_reference():
    # CHUNK_COUNT * 46 / 1000 with integer division (audit/src/lib.rs:955)
    assert audit.CHALLENGE_NEED == 47 and audit.CHUNK_COUNT == 1024


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_challenge_indices_match_oracle(orc, seed):
    rng = np.random.default_rng(seed)
    # a stream with repeats mod 1024 (small values force collisions)
    randoms = rng.integers(0, 2**63, 200, dtype=np.uint64)
    if seed == 1:
        randoms = rng.integers(0, 1100, 400).astype(np.uint64)
    got, used = audit.challenge_indices(randoms)
    want, wused = orc.challenge_indices(randoms.tolist())
    assert got == want and used == wused
    assert len(set(got)) == 47 and all(0 <= i < 1024 for i in got)


def test_challenge_indices_exhausted():
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        audit.challenge_indices([5] * 100)  # one distinct index only


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,F,with_parity", [(2, 1, 8 << 20, True), (2, 1, 1 << 20, False),
                                               (4, 2, 1024 * 48, True), (3, 1, 1024 * 5, True)])
def test_audit_chunks_gpu(k, m, F, with_parity, orc):
    import torch
    import cess_amd
    nseg = 3
    rng = np.random.default_rng(F + k)
    data = rng.integers(0, 256, (nseg, k, F), dtype=np.uint8)
    par = rng.integers(0, 256, (nseg, m, F), dtype=np.uint8)
    idx, _ = audit.challenge_indices(rng.integers(0, 2**63, 400, dtype=np.uint64))
    enc = cess_amd.New(k, m)
    n = k + m if with_parity else k
    chunk = F // 1024
    d_chunks = torch.zeros((nseg * n, len(idx), chunk), dtype=torch.uint8, device="cuda")
    d_hex = torch.zeros((nseg * n, len(idx), 64), dtype=torch.uint8, device="cuda")
    dd, dp = torch.from_numpy(data).cuda(), torch.from_numpy(par).cuda()
    audit.audit_chunks(enc, dd, dp if with_parity else None, nseg, F, idx, d_chunks, d_hex)
    torch.cuda.synchronize()
    got, hx = d_chunks.cpu().numpy(), d_hex.cpu().numpy()
    for f in range(nseg * n):
        s, i = divmod(f, n)
        frag = data[s, i] if i < k else par[s, i - k]
        for j, c in enumerate(idx):
            want = orc.chunk(frag, c)
            assert np.array_equal(got[f, j], want), (f, j)
            assert hx[f, j].tobytes().decode() == hashlib.sha256(want).hexdigest()
    # hashes only (internal scratch for the gathered chunks)
    d_hex2 = torch.zeros_like(d_hex)
    audit.audit_chunks(enc, dd, dp if with_parity else None, nseg, F, idx, None, d_hex2)
    torch.cuda.synchronize()
    assert torch.equal(d_hex, d_hex2)
