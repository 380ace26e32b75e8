"""GPU parity: the HIP path (through the C ABI) against the oracle, bit-exact.

Small sizes compare with the golden fixtures and the C oracle; the full BASELINE geometries
(64 x 16 MiB RS(2,1) segments, 64 x RS(32,32) segments of 512 KiB fragments) compare with the
multi-threaded C oracle and with size-independent properties (encode -> erase -> reconstruct
round trips).
"""
import ctypes
import hashlib

import numpy as np
import pytest

from tests.conftest import case_data, parse_shavs
from oracle.c_oracle import c_encode, ptrs

pytestmark = pytest.mark.gpu

MiB = 1 << 20


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a GPU"
    t.cuda.init()
    return t


@pytest.fixture(scope="module")
def cess(torch):
    import cess_amd
    return cess_amd


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def to_dev(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).cuda()


@pytest.mark.parametrize("generic", [0, 1])
def test_golden_encode_host_api(cess, golden, generic):
    encs = {}
    for case in golden["cases"]:
        k, m = case["k"], case["m"]
        enc = encs.get((k, m))
        if enc is None:
            enc = encs[(k, m)] = cess.New(k, m)
            enc.set_option(1, generic)
        data = case_data(case)
        shards = data + [np.zeros(case["len"], np.uint8) for _ in range(m)]
        enc.Encode(shards)
        assert [sha(p) for p in shards[k:]] == case["parity_sha256"], (k, m, case["len"])
        if "parity_hex" in case:
            assert [p.tobytes().hex() for p in shards[k:]] == case["parity_hex"]
        assert enc.Verify(shards)
        shards[-1][0] ^= 1
        assert not enc.Verify(shards)


@pytest.mark.parametrize("generic", [0, 1])
def test_golden_encode_batch(torch, cess, golden, corc, generic):
    """Batch layout [nseg][k][len]: 3 segments per case (seg s = case data XOR s)."""
    encs = {}
    for case in golden["cases"]:
        k, m, ln = case["k"], case["m"], case["len"]
        enc = encs.get((k, m))
        if enc is None:
            enc = encs[(k, m)] = cess.New(k, m)
            enc.set_option(1, generic)
        base = case_data(case)
        segs = [[(d ^ np.uint8(s)) for d in base] for s in range(3)]
        host = np.stack([np.stack(sg) for sg in segs])  # [3][k][len]
        d_data = to_dev(torch, host)
        d_par = torch.zeros((3, m, ln), dtype=torch.uint8, device="cuda")
        enc.EncodeBatch(d_data, d_par, 3, ln)
        torch.cuda.synchronize()
        got = d_par.cpu().numpy()
        assert [sha(p) for p in got[0]] == case["parity_sha256"]
        for s in range(3):
            want = c_encode(corc, k, m, segs[s])
            for o in range(m):
                assert np.array_equal(got[s, o], want[o]), (k, m, ln, s, o)


@pytest.mark.parametrize("generic", [0, 1])
def test_golden_reconstruct_host_api(cess, golden, corc, generic):
    encs = {}
    for case in golden["cases"]:
        if case["len"] > 1000:
            continue
        k, m = case["k"], case["m"]
        enc = encs.get((k, m))
        if enc is None:
            enc = encs[(k, m)] = cess.New(k, m)
            enc.set_option(1, generic)
        data = case_data(case)
        full = data + c_encode(corc, k, m, data)
        for rec in case["reconstruct"]:
            shards = [None if i in rec["erased"] else full[i].copy() for i in range(k + m)]
            if rec["data_only"]:
                enc.ReconstructData(shards)
            else:
                enc.Reconstruct(shards)
            for i in range(k + m):
                if rec["data_only"] and i >= k and i in rec["erased"]:
                    assert shards[i] is None
                else:
                    assert np.array_equal(shards[i], full[i]), (k, m, rec, i)


@pytest.mark.parametrize("ne", [4, 8, 16, 24, 32])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_host_api_wide_rebuild_reads_only_survivors(cess, corc, ne, mode):
    """The host-buffer API stages only the k survivors (the first k present shards) into HBM, so
    a rebuild must read nothing else: RS(32,32) with shard_len % 1024 == 0 and >= 4 erasures
    runs the FFT-domain decoders (mode 1 / 2 force one), which must take their plans from those
    survivors, not from every shard flagged present (the stage holds stale bytes of the previous
    call there). Every pattern, both data_only settings, bit-exact against the C oracle."""
    k, m, ln = 32, 32, 4096
    rng = np.random.default_rng(100 + ne)
    enc = cess.New(k, m)
    enc.set_option(8, mode)
    for trial in range(6):
        data = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
        full = data + c_encode(corc, k, m, data)
        # a previous call leaves other bytes in the stage: garbage where the next one must not read
        junk = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k + m)]
        enc.Encode(junk)
        erased = set(rng.choice(k + m, size=ne, replace=False).tolist())
        if trial == 0:  # data 0..3 lost plus parity: the advisor's stale-parity pattern
            erased = set(range(min(ne, 4))) | set(range(k + 4, k + 4 + ne - min(ne, 4)))
        for data_only in (False, True):
            shards = [None if i in erased else full[i].copy() for i in range(k + m)]
            (enc.ReconstructData if data_only else enc.Reconstruct)(shards)
            for i in range(k + m):
                if data_only and i >= k and i in erased:
                    assert shards[i] is None
                else:
                    assert np.array_equal(shards[i], full[i]), (ne, mode, trial, data_only, i)


def test_repair_fragment_wide_more_than_k_survivors(cess, corc):
    """repair_fragment with more than k survivors of an RS(32,32) segment that lost many other
    fragments too (a miner exit): the rebuild must come from the staged survivors only."""
    from cess_amd.repair import repair_fragment
    k, m, F = 32, 32, 8192
    rng = np.random.default_rng(8)
    data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
    full = data + c_encode(corc, k, m, data)
    enc = cess.New(k, m)
    for lost in (0, 5, 31, 32, 50):
        others = set(rng.choice([i for i in range(k + m) if i != lost], size=20,
                                replace=False).tolist())
        surv = {i: full[i] for i in range(k + m) if i != lost and i not in others}
        assert len(surv) > k
        got = repair_fragment(enc, surv, lost)
        assert np.array_equal(got, full[lost]), lost


def test_reconstruct_too_few(cess):
    enc = cess.New(4, 2)
    sh = [np.ones(8, np.uint8)] * 6
    with pytest.raises(cess.ErrTooFewShards):
        enc.Reconstruct([None, None, None] + sh[3:])


@pytest.mark.parametrize("k,m,ln,nseg", [(2, 1, 4096, 9), (4, 2, 1000, 7), (32, 32, 4096, 5),
                                         (10, 4, 4099, 6), (2, 1, 1, 3), (2, 1, 4099, 8),
                                         (2, 1, (1 << 16) + 16, 2)])
@pytest.mark.parametrize("generic", [0, 1])
def test_reconstruct_batch_per_segment(torch, cess, corc, k, m, ln, nseg, generic):
    rng = np.random.default_rng(k * 1000 + ln)
    n = k + m
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, n), np.uint8)
    for s in range(nseg):
        if (k, m) == (2, 1):
            present[s, s % 3] = 0  # BASELINE config 3: erased index = seg mod 3
        else:
            e = int(rng.integers(1, m + 1))
            present[s, rng.choice(n, size=e, replace=False)] = 0
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, par * present[:, k:, None])
    enc = cess.New(k, m)
    enc.set_option(1, generic)
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), par)
    # data_only leaves erased parity untouched (still zero)
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, par * present[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present, data_only=True)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), par * present[:, k:, None])


@pytest.mark.parametrize("k,m,ln", [(2, 1, (1 << 16) + 48), (32, 32, (1 << 14) + 4),
                                    (32, 32, 3000 * 4 + 7), (32, 32, 5), (32, 32, 1 << 14),
                                    (32, 32, 96), (32, 32, 3 << 10)])
def test_ct_variants_identical(torch, cess, corc, k, m, ln):
    """Every kernel variant of the tuning build (libcessec_tune.so) is bit-exact too."""
    nseg = 4
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    d_data = to_dev(torch, data)
    enc = cess.New(k, m, tuning=True)
    for v in range(-1, 25):
        enc.set_option(2, v)
        d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
        enc.EncodeBatch(d_data, d_par, nseg, ln)
        torch.cuda.synchronize()
        assert np.array_equal(d_par.cpu().numpy(), want), v
    enc.set_option(2, -1)


@pytest.mark.parametrize("data_only", [0, 1])
def test_mixed21_kargs_variant_leaves_untagged_segments(torch, cess, corc, data_only):
    """Tuning variant 90 (RS(2,1) mixed-pattern rebuild, erasures in the kernel arguments):
    segments with nothing to rebuild are not written (they used to get their parity
    re-encoded, data_only included). Their parity slots hold marker bytes that must survive."""
    k, m, ln, nseg = 2, 1, (1 << 16) + 48, 9
    rng = np.random.default_rng(90)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, 3), np.uint8)
    lost = {0: 0, 1: 1, 3: 0, 4: 2, 7: 1}  # segments 2, 5, 6, 8 intact
    for s, f in lost.items():
        present[s, f] = 0
    marker = par.copy()
    for s in (2, 5, 6, 8):
        marker[s] = 0xA5  # not the codeword's parity: a write would show
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, marker * present[:, k:, None])
    enc = cess.New(k, m, tuning=True)
    enc.set_option(2, 90)
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present, data_only=bool(data_only))
    torch.cuda.synchronize()
    enc.set_option(2, -1)
    assert np.array_equal(d_data.cpu().numpy(), data)
    got = d_par.cpu().numpy()
    for s in range(nseg):
        if s in (2, 5, 6, 8):
            assert (got[s] == 0xA5).all(), s
        elif lost[s] == 2:
            assert np.array_equal(got[s], par[s] if not data_only else 0 * par[s]), s
        else:
            assert np.array_equal(got[s], par[s]), s


@pytest.mark.parametrize("variant", [70, 72, 73, 74, 75, 76, 77, 78, 83, 85, -1])
@pytest.mark.parametrize("nseg,ln", [(1, 4096), (3, 16384), (9, 8192)])
def test_fftdec_d_forms_identical(torch, cess, corc, variant, nseg, ln):
    """The formal-derivative decoder's forms (tuning build): -1 one block per wave (k_fftdec_d,
    the product's), 70 the pipelined persistent kernel (k_fftdec_dp: a wave merges a block's
    output multiplication with the next block's input one), 72 the same with wave priorities, 73
    k_fftdec_d with its quad exchanges through the LDS crossbar (ds_swizzle) in every phase, 74..78
    in some, 83 DPP in every phase through the tuning form, 85 without the skip of unread input
    slots.
    Several segments (per-segment plans), a single segment's host-API-sized batch, 12..32
    erasures: bit-exact with the oracle."""
    k = m = 32
    rng = np.random.default_rng(ln + nseg)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, 64), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(64, size=int(rng.integers(12, 33)), replace=False)] = 0
    enc = cess.New(k, m, tuning=True)
    enc.set_option(2, variant)
    enc.set_option(8, 2)  # the derivative decoder for every segment
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, want * present[:, k:, None])
    before = enc.stat(5)
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert enc.stat(5) - before == nseg
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), want)


@pytest.mark.parametrize("variant", [79, 80, 81, 82, 84, 86, -1])
@pytest.mark.parametrize("nseg,ln,lo,hi", [(1, 4096, 4, 8), (5, 16384, 4, 16), (9, 8192, 9, 20)])
def test_fftdec_m_forms_identical(torch, cess, corc, variant, nseg, ln, lo, hi):
    """The syndrome-row decoder's forms (tuning build): -1 the product's (DPP exchanges), 79..82
    the LDS crossbar for the IFFT's; + the FFT's last layer; + the nibble packs; all three, 84 DPP
    everywhere through the tuning form. Per-segment plans of both
    size classes and both sides (lo..hi erasures): bit-exact with the oracle."""
    k = m = 32
    rng = np.random.default_rng(ln + nseg + lo)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, 64), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(64, size=int(rng.integers(lo, hi + 1)), replace=False)] = 0
    enc = cess.New(k, m, tuning=True)
    enc.set_option(2, variant)
    enc.set_option(8, 1)  # the syndrome-row decoder for every segment
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, want * present[:, k:, None])
    before = enc.stat(4)
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert enc.stat(4) - before == nseg
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), want)


def test_misaligned_layout_byte_path(torch, cess, corc):
    """shard_len % 16 != 0 with nseg > 1 makes shard starts unaligned -> byte kernels."""
    for (k, m) in [(2, 1), (32, 32), (5, 3)]:
        ln, nseg = 1003, 3
        rng = np.random.default_rng(ln + k)
        data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
        want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
        enc = cess.New(k, m)
        d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
        enc.EncodeBatch(to_dev(torch, data), d_par, nseg, ln)
        torch.cuda.synchronize()
        assert np.array_equal(d_par.cpu().numpy(), want)


def test_fill_synthetic_matches_oracle(torch, cess, orc):
    seg_bytes, nseg, seed = 1 << 16, 5, 0xCE550002
    d = torch.empty(nseg * seg_bytes, dtype=torch.uint8, device="cuda")
    cess.fill_synthetic(d, seg_bytes, nseg, 11, seed)
    torch.cuda.synchronize()
    got = d.cpu().numpy().reshape(nseg, seg_bytes)
    for s in range(nseg):
        assert np.array_equal(got[s], orc.synthetic_segment(seed, 11 + s, seg_bytes))


def _full_geometry(torch, cess, corc, k, m, F, nseg, seed):
    seg = k * F
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device="cuda")
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device="cuda")
    cess.fill_synthetic(d_data, seg, nseg, 0, seed)
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, F)
    torch.cuda.synchronize()
    host = d_data.cpu().numpy()
    gpu_par = d_par.cpu().numpy()
    # CPU oracle on the same bytes (all host threads, bounded by 16)
    want = np.zeros_like(gpu_par)
    import os
    corc.orc_encode_batch(k, m, host.ctypes.data, want.ctypes.data, nseg, F,
                          min(16, os.cpu_count() or 1), 1)
    assert np.array_equal(gpu_par, want)
    return enc, d_data, d_par, host, gpu_par


def test_full_geometry_rs21_1gib(torch, cess, corc):
    """BASELINE config 2 + 3 at full size: 64 x 16 MiB segments, then every single erasure."""
    k, m, F, nseg = 2, 1, 8 * MiB, 64
    enc, d_data, d_par, host, par = _full_geometry(torch, cess, corc, k, m, F, nseg, 0xCE550002)
    ref_d, ref_p = d_data.clone(), d_par.clone()
    present = np.ones((nseg, 3), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % 3] = 0
    for s in range(nseg):
        e = s % 3
        if e < k:
            d_data[s, e].zero_()
        else:
            d_par[s, e - k].zero_()
    enc.ReconstructBatch(d_data, d_par, nseg, F, present)
    torch.cuda.synchronize()
    assert torch.equal(d_data, ref_d) and torch.equal(d_par, ref_p)


def test_full_geometry_rs3232(torch, cess, corc):
    """BASELINE config 5 geometry: 64 segments x 32 fragments of 512 KiB, 32 parity each."""
    k, m, F, nseg = 32, 32, 512 * 1024, 64
    enc, d_data, d_par, host, par = _full_geometry(torch, cess, corc, k, m, F, nseg, 0xCE550005)
    ref_d, ref_p = d_data.clone(), d_par.clone()
    rng = np.random.default_rng(3)
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=m, replace=False)] = 0
    pres_t = torch.from_numpy(present).cuda().bool()
    d_data.mul_(pres_t[:, :k, None])
    d_par.mul_(pres_t[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, F, present)
    torch.cuda.synchronize()
    assert torch.equal(d_data, ref_d) and torch.equal(d_par, ref_p)


@pytest.fixture(params=[1, 2, 3], ids=["sha1wave", "sha2wave", "sha_lanepair"])
def sha_mode(request):
    """Run a SHA-256 test with each kernel form (CEC_OPT_SHA_MODE on the test's codec)."""
    return request.param


def test_sha256_shavs_on_gpu(torch, cess, sha_mode):
    """The reference's NIST SHAVS vectors through cec_sha256_batch (one buffer per launch)."""
    vecs = parse_shavs("SHA256ShortMsg.rsp") + parse_shavs("SHA256LongMsg.rsp")
    enc = cess.New(1, 1)
    enc.set_option(3, sha_mode)
    d_hex = torch.zeros((1, 1, 64), dtype=torch.uint8, device="cuda")
    for msg, md in vecs:
        b = torch.from_numpy(np.frombuffer(msg, np.uint8).copy() if msg else
                             np.zeros(1, np.uint8)).cuda()
        enc.Sha256Batch(b, None, 1, len(msg), d_hex)
        torch.cuda.synchronize()
        assert bytes(d_hex.cpu().numpy().reshape(64)).decode() == md, len(msg)


def test_sha256_shavs_pointer_api(torch, cess):
    """cec_sha256_hex (device pointer array, auto kernel) on the SHAVS vectors."""
    vecs = parse_shavs("SHA256ShortMsg.rsp") + parse_shavs("SHA256LongMsg.rsp")
    bufs = [torch.from_numpy(np.frombuffer(msg, np.uint8).copy() if msg else
                             np.zeros(1, np.uint8)).cuda() for msg, _ in vecs]
    for (msg, md), b in zip(vecs, bufs):
        got = cess.sha256_hex_device([b.data_ptr()], len(msg))[0]
        assert got.decode() == md, len(msg)


@pytest.mark.parametrize("length", [0, 1, 55, 56, 63, 64, 119, 120, 1000, 4096 + 17])
def test_sha256_many_unaligned(torch, cess, sha_mode, length):
    """130 buffers (three 64-lane groups, the last partial): back to back in the batch layout
    (odd lengths put every start at a different misalignment) with the chosen kernel form, and
    at odd / 16-byte-aligned starts through the pointer API."""
    n = 130
    rng = np.random.default_rng(length)
    pool = rng.integers(0, 256, n * (length + 32), dtype=np.uint8)
    d_pool = torch.from_numpy(pool).cuda()
    offs = [j * (length + 32) + (j % 5) * 3 for j in range(n)]
    got = cess.sha256_hex_device([d_pool.data_ptr() + o for o in offs], length)
    for j, o in enumerate(offs):
        assert got[j].decode() == sha(pool[o:o + length]), j
    enc = cess.New(1, 1)
    enc.set_option(3, sha_mode)
    d_hex = torch.zeros((n, 1, 64), dtype=torch.uint8, device="cuda")
    enc.Sha256Batch(d_pool, None, n, length, d_hex)
    torch.cuda.synchronize()
    hx = d_hex.cpu().numpy().reshape(n, 64)
    for j in range(n):
        assert hx[j].tobytes().decode() == sha(pool[j * length:(j + 1) * length]), j


def test_sha256_batch_matches_hashlib(torch, cess, sha_mode):
    for (k, m, F, nseg) in [(2, 1, 4096 + 7, 3), (32, 32, 65536, 2), (2, 1, 1 << 20, 4)]:
        rng = np.random.default_rng(F)
        data = rng.integers(0, 256, (nseg, k, F), dtype=np.uint8)
        par = rng.integers(0, 256, (nseg, m, F), dtype=np.uint8)
        enc = cess.New(k, m)
        d_hex = torch.zeros((nseg, k + m, 64), dtype=torch.uint8, device="cuda")
        enc.Sha256Batch(to_dev(torch, data), to_dev(torch, par), nseg, F, d_hex)
        torch.cuda.synchronize()
        hx = d_hex.cpu().numpy()
        for s in range(nseg):
            for i in range(k + m):
                buf = data[s, i] if i < k else par[s, i - k]
                assert hx[s, i].tobytes().decode() == sha(buf)


@pytest.mark.parametrize("size,seg,k,m,hash_on,window", [
    (3 * (1 << 20) + 12345, 1 << 20, 2, 1, "host", 32),
    (7 * (1 << 19) + 1, 1 << 19, 4, 2, "host", 1),
    (11 * 3000 + 17, 3000, 3, 2, "host", 1),         # F = 1000: no prefix digest (F % 64 != 0)
    (5 * (1 << 20) + 7, 1 << 20, 2, 1, "gpu", 32),
    (9 * (1 << 20) + 7, 1 << 20, 2, 1, "gpu", 2),   # device slots reused (5 batches, window 2)
    (7 * (1 << 19) + 1, 1 << 19, 4, 2, "gpu", 1),
    (2 * (1 << 20) - 5, 1 << 19, 32, 32, "auto", 32),
    (40 * MiB + 3, 16 * MiB, 2, 1, "auto", 32),
])
def test_segment_list_pipeline(torch, cess, orc, size, seg, k, m, hash_on, window):
    """§8f rank 1: file -> segments -> fragments -> SegmentList, vs the oracle."""
    from cess_amd.segments import SegmentEncoder, check_file_spec, needed_space
    rng = np.random.default_rng(size)
    blob = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    se = SegmentEncoder(k, m, seg, batch_segments=2, hash_on=hash_on, window=window)
    frags = {}
    rec = se.encode_file(blob, on_fragment=lambda s, i, b: frags.__setitem__((s, i), sha(b)))
    se.close()
    want = orc.segment_list(blob, k, m, seg)
    assert [(s.hash, s.fragment_list) for s in rec.segments] == want
    assert rec.file_hash == orc.file_hash(want)
    assert rec.size == size
    assert check_file_spec(rec.segments, k + m)
    assert needed_space(rec.segments, seg) == len(want) * seg * 15 // 10
    for (s, i), h in frags.items():
        assert h.encode() == want[s][1][i]


def test_segment_list_auto_placement(torch, cess, orc, monkeypatch):
    """hash_on="auto" re-places hashing per file by size (host below AUTO_GPU_BYTES, GPU hash
    queue above) on one encoder, records identical either way."""
    from cess_amd.segments import SegmentEncoder
    monkeypatch.setattr(SegmentEncoder, "AUTO_GPU_BYTES", 3 << 20)
    seg = 1 << 20
    se = SegmentEncoder(2, 1, seg, batch_segments=2, hash_on="auto", window=2)
    for size, want_on in [((2 << 20) + 5, "host"), ((7 << 20) + 3, "gpu"), (1 << 20, "host"),
                          (5 << 20, "gpu")]:
        blob = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8)
        rec = se.encode_file(blob)
        assert se.hash_on == want_on
        want = orc.segment_list(blob.tobytes(), 2, 1, seg)
        assert [(s_.hash, s_.fragment_list) for s_ in rec.segments] == want
    se.close()


@pytest.mark.parametrize("k,m,exchange", [(2, 1, "survivors"), (2, 1, "partials"),
                                          (10, 4, "partials"), (10, 4, "auto")])
def test_degraded_read_single_rank(torch, cess, corc, k, m, exchange):
    """distributed.degraded_read end to end on one GPU (world 1: every survivor is local, so
    no P2P op is issued; the decode runs through libcessec). With the partial-product exchange
    the decoder holds every survivor: its own partial is the whole rebuild, nothing to XOR."""
    from cess_amd import distributed as D
    F, nseg = 1 << 16, 6
    rng = np.random.default_rng(11)
    full = []
    for s in range(nseg):
        data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
        full.append(data + c_encode(corc, k, m, data))
    mine = D.local_fragments(nseg, k + m, 1, 0)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).cuda())
    lost = {s: [s % (k + m)] for s in range(nseg)}
    plan = D.plan_gather(lost, k, m, 1, F, exchange=exchange)
    assert plan.bytes_moved == 0
    assert bool(plan.partial) == (exchange == "partials")
    out = D.degraded_read(plan, store, cess.New(k, m), 0)
    torch.cuda.synchronize()
    assert len(out) == nseg
    for (s, f), t in out.items():
        assert np.array_equal(t.cpu().numpy(), full[s][f])


def test_max_shards_256(cess, corc):
    """k + m = 256 (the GF(2^8) limit): run-time kernel, outputs split over chunks of 32."""
    k, m, ln = 200, 56, 272
    rng = np.random.default_rng(256)
    data = [rng.integers(0, 256, ln, dtype=np.uint8) for _ in range(k)]
    want = c_encode(corc, k, m, data)
    enc = cess.New(k, m)
    shards = data + [np.zeros(ln, np.uint8) for _ in range(m)]
    enc.Encode(shards)
    assert all(np.array_equal(a, b) for a, b in zip(shards[k:], want))
    erased = set(rng.choice(k + m, size=m, replace=False).tolist())
    full = data + want
    sh = [None if i in erased else full[i].copy() for i in range(k + m)]
    enc.Reconstruct(sh)
    assert all(np.array_equal(a, b) for a, b in zip(sh, full))
    with pytest.raises(cess.ErrMaxShardNum):
        cess.New(200, 57)


@pytest.mark.parametrize("k,m", [(1, 255), (255, 1), (128, 128), (3, 253), (253, 3)])
def test_extreme_codes_batched(torch, cess, corc, k, m):
    """Codes at the GF(2^8) limit k + m = 256 with one data shard, one parity shard or an even
    split: batched encode equal to the C oracle, and a rebuild of m random erasures (every one
    of the erasable count) per segment restoring the oracle's codeword."""
    ln, nseg = 1000 + 3, 2
    rng = np.random.default_rng(k * 1000 + m)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, [data[s, i] for i in range(k)]))
                     for s in range(nseg)])
    enc = cess.New(k, m)
    d_data = to_dev(torch, data)
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc.EncodeBatch(d_data, d_par, nseg, ln)
    torch.cuda.synchronize()
    assert np.array_equal(d_par.cpu().numpy(), want)
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=m, replace=False)] = 0
    dd, dp = d_data.clone(), d_par.clone()
    for s in range(nseg):
        for f in np.flatnonzero(present[s] == 0):
            (dd[s, f] if f < k else dp[s, f - k]).fill_(0xA5)
    enc.ReconstructBatch(dd, dp, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(dd.cpu().numpy(), data)
    assert np.array_equal(dp.cpu().numpy(), want)
    enc.close()


def test_more_segments_than_grid_y(torch, cess, corc):
    """nseg > 65535 splits the launch over grid.y chunks (encode, verify, per-segment decode)."""
    k, m, ln, nseg = 2, 1, 32, 70000
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    d_data = to_dev(torch, data)
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, ln)
    torch.cuda.synchronize()
    par = d_par.cpu().numpy()
    want = np.zeros_like(par)
    corc.orc_encode_batch(k, m, data.ctypes.data, want.ctypes.data, nseg, ln, 8, 1)
    assert np.array_equal(par, want)
    d_par[nseg - 2, 0, 5] ^= 1  # one bad segment in the last grid.y chunk
    for generic in (0, 1):
        enc.set_option(1, generic)
        ok = enc.VerifyBatch(d_data, d_par, nseg, ln)
        assert ok.sum() == nseg - 1 and not ok[nseg - 2], generic
    enc.set_option(1, 0)
    present = np.ones((nseg, 3), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % 3] = 0
    for generic in (0, 1):
        enc.set_option(1, generic)
        dd = to_dev(torch, data * present[:, :k, None])
        dp = to_dev(torch, want * present[:, k:, None])
        enc.ReconstructBatch(dd, dp, nseg, ln, present)
        torch.cuda.synchronize()
        assert np.array_equal(dd.cpu().numpy(), data) and np.array_equal(dp.cpu().numpy(), want)


def test_fft_more_segments_than_grid_y(torch, cess, corc):
    """RS(32,32) (the FFT encode and the fused FFT verify) over 70,000 segments of 1 KiB
    fragments: segments either side of each grid.y chunk boundary match the C oracle, and one
    corrupted segment in the last chunk is the only one that fails verification."""
    k, m, ln, nseg = 32, 32, 1024, 70000
    gen = torch.Generator(device="cuda").manual_seed(5)
    d_data = torch.randint(0, 256, (nseg, k, ln), dtype=torch.uint8, device="cuda", generator=gen)
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, ln)
    torch.cuda.synchronize()
    for s in (0, 65534, 65535, nseg - 1):
        want = np.stack(c_encode(corc, k, m, list(d_data[s].cpu().numpy())))
        assert np.array_equal(d_par[s].cpu().numpy(), want), s
    assert enc.VerifyBatch(d_data, d_par, nseg, ln).all()
    d_data[nseg - 3, 31, ln - 1] ^= 0x80
    ok = enc.VerifyBatch(d_data, d_par, nseg, ln)
    assert ok.sum() == nseg - 1 and not ok[nseg - 3]


def test_fftdec_more_segments_than_grid_y(torch, cess):
    """The FFT-domain decoders over 70,000 RS(32,32) segments of 1 KiB fragments: one pattern for
    the whole batch, then per-segment patterns cycling over both sides and both size classes
    (launches split at grid.y chunks, plans indexed per listed segment); every segment equals the
    encoded original."""
    k, m, ln, nseg = 32, 32, 1024, 70000
    gen = torch.Generator(device="cuda").manual_seed(6)
    d_data = torch.randint(0, 256, (nseg, k, ln), dtype=torch.uint8, device="cuda", generator=gen)
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, ln)
    ref_d, ref_p = d_data.clone(), d_par.clone()
    rng = np.random.default_rng(70)
    pats = []
    for ne, lo, hi in ((8, 0, 64), (6, 0, 32), (6, 32, 64), (16, 0, 64), (12, 0, 64)):
        p = np.ones(64, np.uint8)
        p[lo + rng.choice(hi - lo, size=ne, replace=False)] = 0
        pats.append(p)
    before = enc.stat(4)
    try:
        for mode, per_seg in ((1, False), (1, True), (2, False), (2, True)):
            enc.set_option(8, mode)  # every pattern on that decoder (syndrome rows / derivative)
            present = np.stack([pats[s % len(pats)] for s in range(nseg)]) if per_seg else pats[0]
            pm = torch.from_numpy(present if per_seg else present[None].repeat(nseg, 0)).cuda()
            d_data.mul_(pm[:, :k, None])
            d_par.mul_(pm[:, k:, None])
            enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
            torch.cuda.synchronize()
            assert torch.equal(d_data, ref_d) and torch.equal(d_par, ref_p), (mode, per_seg)
        assert enc.stat(4) - before == 4 * nseg
    finally:
        enc.set_option(8, 0)


def test_encode_file_sharded_single_rank(tmp_path, orc):
    from cess_amd.segments import encode_file_sharded
    rng = np.random.default_rng(21)
    blob = rng.integers(0, 256, 5 * MiB + 77, dtype=np.uint8).tobytes()
    p = tmp_path / "g.bin"
    p.write_bytes(blob)
    for world_slice in range(3):  # each rank's range on its own, as a world of 3 would do
        from cess_amd.distributed import shard_range
        a, b = shard_range(6, 3, world_slice)
        from cess_amd.segments import SegmentEncoder
        se = SegmentEncoder(2, 1, 1 << 20, batch_segments=2)
        rec = se.encode_range(str(p), a, b)
        se.close()
        want = orc.segment_list(blob, 2, 1, 1 << 20)[a:b]
        assert [(s.hash, s.fragment_list) for s in rec.segments] == want
    from cess_amd.pipeline import RecordsSession
    for hash_on in ("hybrid", "host", "gpu"):
        with RecordsSession(2, 1, 1 << 20, 0, hash_on, batch_segments=2) as ses:
            for world_slice in range(3):
                a, b = shard_range(6, 3, world_slice)
                want = orc.segment_list(blob, 2, 1, 1 << 20)[a:b]
                for src in (str(p), np.frombuffer(blob, np.uint8)):
                    rec, _ = ses.encode_range(src, a, b)
                    assert [(s.hash, s.fragment_list) for s in rec.segments] == want, hash_on
                    assert rec.file_hash == orc.file_hash(want)
    rec = encode_file_sharded(str(p), 0, 1, segment_size=1 << 20, batch_segments=4)
    assert [(s.hash, s.fragment_list) for s in rec.segments] == orc.segment_list(
        blob, 2, 1, 1 << 20)
    assert rec.file_hash == orc.file_hash(orc.segment_list(blob, 2, 1, 1 << 20))


def test_repair_fragment_and_hash_check(cess, corc, orc):
    """§8f rank 2: restoral — rebuild one fragment from peer survivors, check the recorded hash."""
    from cess_amd.repair import ErrFragmentHashMismatch, repair_fragment
    k, m, F = 2, 1, 1 << 20
    rng = np.random.default_rng(5)
    data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
    full = data + c_encode(corc, k, m, data)
    hashes = [orc.sha256_hex(x) for x in full]
    enc = cess.New(k, m)
    for lost in range(3):
        surv = {i: full[i] for i in range(3) if i != lost}
        got = repair_fragment(enc, surv, lost, hashes[lost])
        assert np.array_equal(got, full[lost])
    bad = {0: full[0], 2: full[2].copy()}
    bad[2][7] ^= 1
    with pytest.raises(ErrFragmentHashMismatch):
        repair_fragment(enc, bad, 1, hashes[1])
    with pytest.raises(cess.ErrTooFewShards):
        repair_fragment(enc, {0: full[0]}, 1)


def test_repair_batch_wide(torch, cess, corc, orc):
    from cess_amd.repair import repair_batch
    k, m, F, nseg = 10, 4, 4096, 5
    rng = np.random.default_rng(6)
    data = rng.integers(0, 256, (nseg, k, F), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, k + m), np.uint8)
    expected = []
    for s in range(nseg):
        lost = rng.choice(k + m, size=1 + s % m, replace=False)
        present[s, lost] = 0
        expected.append({int(i): orc.sha256_hex(data[s, i] if i < k else par[s, i - k])
                         for i in lost})
    dd = to_dev(torch, data * present[:, :k, None])
    dp = to_dev(torch, par * present[:, k:, None])
    enc = cess.New(k, m)
    # a recorded hash that the rebuilt fragment does not match flags that segment only
    wrong = [dict(e) for e in expected]
    i0 = next(iter(wrong[2]))
    wrong[2][i0] = b"0" * 64
    for hash_on in ("gpu", "host", "auto"):  # the check on the GPU or on host cores
        ok = repair_batch(enc, dd, dp, nseg, F, present, expected, hash_on=hash_on)
        assert ok == [True] * nseg, hash_on
        assert repair_batch(enc, dd, dp, nseg, F, present, wrong, hash_on=hash_on) == \
            [True, True, False, True, True], hash_on
    with pytest.raises(ValueError):
        repair_batch(enc, dd, dp, nseg, F, present, expected, hash_on="tpu")


def test_repair_batch_host_check_ring(torch, cess, corc, orc):
    """The host-side check copies the rebuilt fragments out through a ring of pinned chunks
    (repair.CHECK_RING x CHECK_CHUNK): a batch of many more fragments than the ring holds, with
    a ragged last chunk and one wrong recorded hash deep in the batch."""
    from cess_amd import repair
    k, m, F, nseg = 2, 1, 4096 + 64, repair.CHECK_RING * repair.CHECK_CHUNK * 2 + 7
    rng = np.random.default_rng(16)
    data = rng.integers(0, 256, (nseg, k, F), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, k + m), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % 3] = 0
    expected = [{s % 3: orc.sha256_hex(data[s, s % 3] if s % 3 < k else par[s, 0])}
                for s in range(nseg)]
    expected[nseg - 20] = {(nseg - 20) % 3: b"f" * 64}
    dd = to_dev(torch, data * present[:, :k, None])
    dp = to_dev(torch, par * present[:, k:, None])
    enc = cess.New(k, m)
    ok = repair.repair_batch(enc, dd, dp, nseg, F, present, expected, hash_on="host")
    assert ok == [s != nseg - 20 for s in range(nseg)]


def test_repair_emits_completion_only_for_matching_hash(torch, cess, corc, orc):
    """The repair service reports a rebuilt fragment with restoral_order_complete(fragment_hash)
    (call 16, c-pallets/file-bank/src/lib.rs:1072-1122) only when its SHA-256 matched the
    recorded hash: a segment whose rebuild does not match yields no completion call."""
    from cess_amd import records
    from cess_amd.repair import ErrFragmentHashMismatch, repair_batch, repair_fragment
    k, m, F, nseg = 2, 1, 1 << 16, 6
    rng = np.random.default_rng(8)
    data = rng.integers(0, 256, (nseg, k, F), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, k + m), np.uint8)
    expected = []
    for s in range(nseg):
        present[s, s % 3] = 0
        i = s % 3
        expected.append({i: orc.sha256_hex(data[s, i] if i < k else par[s, i - k])})
    dd = to_dev(torch, data * present[:, :k, None])
    dp = to_dev(torch, par * present[:, k:, None])
    dp_corrupt = dp.clone()
    enc = cess.New(k, m)
    # segment 4 lost data fragment 1; its surviving parity is corrupted -> rebuilt bytes differ
    dp_corrupt[4, 0, 100] ^= 0x40
    for hash_on in ("gpu", "host"):
        ok, calls = repair_batch(enc, dd.clone(), dp.clone(), nseg, F, present, expected,
                                 hash_on=hash_on, complete_calls=True)
        assert ok == [True] * nseg
        assert calls == {(s, s % 3): records.restoral_order_complete(expected[s][s % 3])
                         for s in range(nseg)}
        ok, calls = repair_batch(enc, dd.clone(), dp_corrupt.clone(), nseg, F, present,
                                 expected, hash_on=hash_on, complete_calls=True)
        assert ok == [s != 4 for s in range(nseg)], hash_on
        assert (4, 1) not in calls and len(calls) == nseg - 1
        assert all(c == bytes([60, 16]) + expected[s][i] for (s, i), c in calls.items())
    full = [data[0, 0], data[0, 1], par[0, 0]]
    frag, call = repair_fragment(enc, {1: full[1], 2: full[2]}, 0, expected[0][0],
                                 complete_call=True)
    assert np.array_equal(frag, full[0]) and call == records.restoral_order_complete(expected[0][0])
    bad = full[2].copy()
    bad[0] ^= 1
    with pytest.raises(ErrFragmentHashMismatch):  # no call data on a mismatch
        repair_fragment(enc, {1: full[1], 2: bad}, 0, expected[0][0], complete_call=True)


def test_filler_upload_records(torch, orc):
    """Idle fillers with their on-chain records: FillerInfo { block_num, miner_address,
    filler_hash } (types.rs:82-86) from the GPU filler hashes, UploadFillerLimit = 10 per
    upload_filler call (lib.rs:795-833, runtime/src/lib.rs:1033)."""
    import struct
    from cess_amd import records
    from cess_amd.repair import generate_filler_upload
    miner, tee = bytes(range(32)), bytes(range(100, 132))
    d, hashes, fillers, calls = generate_filler_upload(12, miner, tee, block_num=77, first=3)
    assert d.shape == (12, 8 << 20) and len(calls) == 2
    for i in (0, 11):
        want = orc.synthetic_segment(0xF111E5, 3 + i, 8 << 20)
        assert hashes[i] == orc.sha256_hex(want)
    assert [f.filler_hash for f in fillers] == hashes
    assert calls[0] == bytes([60, 8]) + tee + bytes([10 << 2]) + b"".join(
        struct.pack("<I", 77) + miner + h for h in hashes[:10])
    assert calls[1] == records.upload_filler(tee, fillers[10:])


@pytest.mark.parametrize("hash_on", ["auto", "gpu", "host"])
def test_generate_fillers(torch, orc, hash_on):
    from cess_amd.repair import generate_fillers
    n = 3 if hash_on != "host" else 40  # the host path through more than two pinned chunks
    d, hashes = generate_fillers(n, filler_size=1 << 16, first=7, hash_on=hash_on)
    for i in range(n):
        want = orc.synthetic_segment(0xF111E5, 7 + i, 1 << 16)
        assert np.array_equal(d[i].cpu().numpy(), want)
        assert hashes[i] == orc.sha256_hex(want)


def test_c_abi_consumer(tmp_path):
    """A plain C program against include/cess_ec.h (no Python): encode, verify, every single
    erasure rebuilt, error codes — what a cgo/FFI binding exercises."""
    import subprocess
    from tests.conftest import ROOT
    exe = tmp_path / "cabi_roundtrip"
    lib = f"{ROOT}/cess_amd"
    orc = f"{ROOT}/oracle/build"
    subprocess.run(["gcc", "-O2", f"{ROOT}/tests/native/cabi_roundtrip.c", f"-I{ROOT}/include",
                    f"-L{lib}", "-lcessec", f"-L{orc}", "-loracle",
                    f"-Wl,-rpath,{lib}:{orc}", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "cabi roundtrip ok" in r.stdout


@pytest.mark.parametrize("k,m,ln,ne", [(32, 32, 4096 + 3, 32), (10, 4, 1000, 4),
                                       (17, 3, 4099, 3), (33, 3, 515, 3), (1, 1, 9, 1),
                                       (5, 5, 64, 5), (32, 32, 4096 + 3, 1),
                                       (32, 32, (1 << 16) + 16, 2), (10, 4, 4099, 1),
                                       (32, 32, 4096 + 3, 6), (32, 32, (1 << 16) + 16, 8),
                                       (20, 10, 999, 5)])
def test_runtime_kernels_agree(torch, cess, corc, k, m, ln, ne):
    """k_rth (Horner over input groups, run-time indices), k_rt (per-bit masks), k_rthx
    (Horner with index-mode XORs) and k_rtb (bit-plane accumulators, chunks of <= 4 outputs)
    against the C oracle: encode and per-segment reconstruct of `ne` random erasures, vector body
    and byte tail."""
    nseg = 3
    rng = np.random.default_rng(k * 1000 + ln + ne)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=ne, replace=False)] = 0
    enc = cess.New(k, m)
    enc.set_option(1, 1)  # run-time coefficients for encode too
    try:
        for mode in (0, 1, 2, 3):
            enc.set_option(4, mode)
            d_data = to_dev(torch, data)
            d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
            enc.EncodeBatch(d_data, d_par, nseg, ln)
            torch.cuda.synchronize()
            assert np.array_equal(d_par.cpu().numpy(), want), ("encode", mode)
            keep = torch.from_numpy(present[:, :k, None].astype(np.uint8)).cuda()
            keep_p = torch.from_numpy(present[:, k:, None].astype(np.uint8)).cuda()
            d_data *= keep
            d_par *= keep_p
            enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
            torch.cuda.synchronize()
            assert np.array_equal(d_data.cpu().numpy(), data), ("reconstruct", mode)
            assert np.array_equal(d_par.cpu().numpy(), want), ("reconstruct parity", mode)
    finally:
        enc.set_option(4, 0)


def _wide_patterns(rng, nseg, ne):
    """RS(32,32) erasure patterns: random, all on one coset, split evenly, per segment."""
    present = np.ones((nseg, 64), np.uint8)
    for s in range(nseg):
        kind = s % 4
        if kind == 0 or ne > 32:
            present[s, rng.choice(64, size=ne, replace=False)] = 0
        elif kind == 1:  # data only lost (the side with more erasures is data)
            present[s, rng.choice(32, size=min(ne, 32), replace=False)] = 0
        elif kind == 2:  # parity mostly
            present[s, 32 + rng.choice(32, size=min(ne, 32), replace=False)] = 0
        else:  # half and half
            a = ne // 2
            present[s, rng.choice(32, size=a, replace=False)] = 0
            present[s, 32 + rng.choice(32, size=ne - a, replace=False)] = 0
    return present


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("ne", [2, 3, 5, 8, 13, 16, 24, 31, 32])
@pytest.mark.parametrize("ln", [1024, 8192, 3 * 1024 + 512 * 2])
def test_fftdec_matches_oracle(torch, cess, corc, ne, ln, mode):
    """RS(32,32) rebuilds on the FFT-domain erasure decoders (mode 1, fftdec.hip: T1 transform,
    syndromes, bit-plane run-time rows; mode 2, fftdec_d.hip: the formal-derivative decoder over
    64-point transforms) are bit-exact with the C oracle's codeword: per-segment patterns on both
    sides (data / parity / mixed erasures), one pattern for the whole batch, data_only, and the
    same bytes as the run-time matrix kernels (CEC_OPT_FFTDEC_MIN = 0)."""
    k = m = 32
    nseg = 8
    rng = np.random.default_rng(ne * 7 + ln)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = _wide_patterns(rng, nseg, ne)
    enc = cess.New(k, m)
    enc.set_option(8, mode)  # every FFT-domain-eligible rebuild on that decoder (no cost model)
    before = enc.stat(4)
    for fmin in (2, 0):  # the FFT-domain decoder from two outputs, then never
        enc.set_option(7, fmin)
        d_data = to_dev(torch, data * present[:, :k, None])
        d_par = to_dev(torch, want * present[:, k:, None])
        enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
        torch.cuda.synchronize()
        assert np.array_equal(d_data.cpu().numpy(), data), ("per-segment data", fmin)
        assert np.array_equal(d_par.cpu().numpy(), want), ("per-segment parity", fmin)
        # one pattern for every segment, and data_only (parity stays erased)
        one = present[3]
        d_data = to_dev(torch, data * one[None, :k, None])
        d_par = to_dev(torch, want * one[None, k:, None])
        enc.ReconstructBatch(d_data, d_par, nseg, ln, one, data_only=True)
        torch.cuda.synchronize()
        assert np.array_equal(d_data.cpu().numpy(), data), ("data_only", fmin)
        assert np.array_equal(d_par.cpu().numpy(), want * one[None, k:, None]), ("data_only p", fmin)
        if fmin:  # the per-segment call ran on the decoder (data_only may leave < 2 outputs)
            assert enc.stat(4) - before >= nseg, mode
    enc.set_option(7, 4)
    enc.set_option(8, 0)


@pytest.mark.parametrize("ln,nd_want", [(512 * 1024, 2), (2048, 8)])
def test_fftdec_both_decoders_one_call(torch, cess, corc, ln, nd_want):
    """One per-segment rebuild whose patterns the cost model sends 6 segments to the syndrome-row
    decoder (8 erasures) and 2 to the formal-derivative decoder (32). At 512 KiB shards the split
    pays for its second launch: both launches write their own segments only, bit-exact with the C
    oracle. At 2 KiB the whole batch is cheaper on the derivative decoder alone (the batch-level
    split rule folds the syndrome-row segments into its launch)."""
    k = m = 32
    nseg = 8
    rng = np.random.default_rng(808)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, 64), np.uint8)
    for s in range(nseg):
        if s in (2, 5):
            present[s, rng.choice(64, size=32, replace=False)] = 0
        else:  # one pattern: data 0-3 and parity 32-35 lost (one syndrome-row launch class)
            present[s, [0, 1, 2, 3, 32, 33, 34, 35]] = 0
    enc = cess.New(k, m)
    b4, b5 = enc.stat(4), enc.stat(5)
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, want * present[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), want)
    assert enc.stat(4) - b4 == nseg and enc.stat(5) - b5 == nd_want


@pytest.mark.parametrize("ln", [1000, 1024 + 512])
def test_fftdec_d_layout_fallback(torch, cess, corc, ln):
    """A layout the FFT-domain decoders cannot take (shard_len % 1024 != 0) with the
    formal-derivative decoder forced (CEC_OPT_FFTDEC_MODE 2): the rebuild runs the run-time matrix
    kernels instead, bit-exact, and CEC_STAT_FFTDEC_D_SEGMENTS does not move."""
    k = m = 32
    nseg = 4
    rng = np.random.default_rng(ln)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = _wide_patterns(rng, nseg, 32)
    enc = cess.New(k, m)
    enc.set_option(8, 2)
    before = enc.stat(5)
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, want * present[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), want)
    assert enc.stat(5) == before


@pytest.mark.parametrize("ne", [8, 32])
def test_fftdec_dispatch_by_cost(torch, cess, corc, ne):
    """CEC_OPT_FFTDEC_MODE 0 (the default) sends a random RS(32,32) pattern to the cheapest of the
    FFT-domain decoders and k_rthx by the cost model (eight erasures: the syndrome-row decoder; 32
    with 16 syndrome slots: the formal-derivative decoder, no longer the matrix kernel), counted by
    CEC_STAT_FFTDEC_SEGMENTS; bit-exact either way."""
    k = m = 32
    nseg, ln = 6, 4096
    rng = np.random.default_rng(500 + ne)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, 64), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(32, size=ne // 2, replace=False)] = 0
        if ne == 32:  # every even parity shard: the 16 syndrome rows sit in 16 slots
            present[s, 32::2] = 0
        else:
            present[s, 32 + rng.choice(32, size=ne - ne // 2, replace=False)] = 0
    enc = cess.New(k, m)
    before, before_d = enc.stat(4), enc.stat(5)
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, want * present[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), want)
    on_fd, on_d = enc.stat(4) - before, enc.stat(5) - before_d
    assert on_fd == nseg, on_fd
    assert on_d == (nseg if ne == 32 else 0), on_d  # 32: the derivative decoder; 8: syndrome rows


@pytest.mark.parametrize("ne,ln", [(1, 4096 + 3), (2, (1 << 16) + 16), (3, 4096 + 3), (4, 999)])
def test_rtb_tuning_shapes_agree(torch, cess, corc, ne, ln):
    """The tuning build's k_rtb shapes (column width x columns in flight, variants 40-49)
    rebuild RS(32,32) erasures bit-exact: vector body and byte tail."""
    k, m, nseg = 32, 32, 3
    rng = np.random.default_rng(77 + ne)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=ne, replace=False)] = 0
    enc = cess.New(k, m, tuning=True)
    enc.set_option(4, 3)
    enc.set_option(7, 0)  # the bit-plane kernel, never the FFT-domain decoder
    for v in [-1] + list(range(40, 50)):
        enc.set_option(2, v)
        d_data = to_dev(torch, data * present[:, :k, None])
        d_par = to_dev(torch, want * present[:, k:, None])
        enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
        torch.cuda.synchronize()
        assert np.array_equal(d_data.cpu().numpy(), data), v
        assert np.array_equal(d_par.cpu().numpy(), want), v



@pytest.mark.parametrize("k,m,ln", [(32, 32, 4096 + 4), (10, 4, 1000)])
def test_decode_cache_eviction(torch, cess, corc, k, m, ln):
    """The decode-program LRU cache at capacity 8 (CEC_OPT_DECODE_CACHE) under per-segment
    ReconstructBatch calls with 24 distinct erasure patterns each: programs resolved early in a
    call stay valid while later patterns push the cache past its cap, and retired device blocks
    are reused only after the launches that read them (bit-exact vs the C oracle every call)."""
    nseg, ncall = 24, 3
    n = k + m
    rng = np.random.default_rng(k * 7 + ln)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    enc = cess.New(k, m)
    enc.set_option(6, 8)
    for call in range(ncall):
        present = np.ones((nseg, n), np.uint8)
        seen = set()
        for s in range(nseg):
            while True:
                e = rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)
                key = tuple(sorted(e.tolist()))
                if key not in seen:
                    seen.add(key)
                    break
            present[s, list(key)] = 0
        d_data = to_dev(torch, data * present[:, :k, None])
        d_par = to_dev(torch, par * present[:, k:, None])
        enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
        assert enc.stat(1) <= 8  # CEC_STAT_DECODE_CACHED
        torch.cuda.synchronize()
        assert np.array_equal(d_data.cpu().numpy(), data), call
        assert np.array_equal(d_par.cpu().numpy(), par), call


def test_back_to_back_plans_on_side_stream(torch, cess, corc):
    """Per-segment reconstructs with different pattern maps enqueued back to back on a
    non-blocking side stream without host synchronisation: each call's plan (segment list,
    chunk pointers) must not be overwritten while earlier launches still read it."""
    k, m, ln, nseg = 10, 4, 1 << 16, 16
    n = k + m
    rng = np.random.default_rng(99)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    enc = cess.New(k, m)
    enc.set_option(6, 4)
    calls = []
    for _ in range(6):
        present = np.ones((nseg, n), np.uint8)
        for s in range(nseg):
            present[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 0
        calls.append((present, to_dev(torch, data * present[:, :k, None]),
                      to_dev(torch, par * present[:, k:, None])))
    torch.cuda.synchronize()  # inputs in place; from here the calls only enqueue
    side = torch.cuda.Stream()
    for present, d_data, d_par in calls:
        enc.ReconstructBatch(d_data, d_par, nseg, ln, present, stream=side)
    side.synchronize()
    for present, d_data, d_par in calls:
        assert np.array_equal(d_data.cpu().numpy(), data)
        assert np.array_equal(d_par.cpu().numpy(), par)


def test_full_geometry_config4_64gib(torch, cess, corc):
    """BASELINE config 4 at world 1: the 64 GiB file (4096 x 16 MiB segments) encoded in one
    batch in HBM (64 GiB data + 32 GiB parity); 8 sampled segments against the C oracle, then
    the round-trip property on every segment: erase fragment s mod 3 of each, rebuild all 4096
    in one per-segment call, compare with the erased originals (kept in HBM)."""
    k, m, F, nseg = 2, 1, 8 * MiB, 4096
    free, _ = torch.cuda.mem_get_info()
    if free < (140 << 30):
        pytest.skip(f"needs ~140 GiB of free HBM, {free >> 30} GiB free")
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device="cuda")
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device="cuda")
    cess.fill_synthetic(d_data, k * F, nseg, 0, 0xCE550004)
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, F)
    torch.cuda.synchronize()
    sample = [0, 1, 777, 1500, 2048, 3001, 4094, 4095]
    host = d_data[sample].cpu().numpy()
    want = np.zeros((len(sample), m, F), np.uint8)
    corc.orc_encode_batch(k, m, host.ctypes.data, want.ctypes.data, len(sample), F, 8, 1)
    assert np.array_equal(d_par[sample].cpu().numpy(), want)
    # keep the fragment each segment loses (32 GiB), erase it, rebuild everything at once
    seg = torch.arange(nseg, device="cuda")
    lost = seg % 3
    keep = torch.empty((nseg, F), dtype=torch.uint8, device="cuda")
    for e in range(3):
        idx = seg[lost == e]
        src = d_data[idx, e] if e < k else d_par[idx, e - k]
        keep[idx] = src
        if e < k:
            d_data[idx, e] = 0
        else:
            d_par[idx, e - k] = 0
    present = np.ones((nseg, k + m), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % 3] = 0
    enc.ReconstructBatch(d_data, d_par, nseg, F, present)
    torch.cuda.synchronize()
    for e in range(3):
        idx = seg[lost == e]
        got = d_data[idx, e] if e < k else d_par[idx, e - k]
        assert torch.equal(got, keep[idx]), e


def test_config1_single_segment_host_api(cess, corc):
    """BASELINE config 1's workload through the klauspost-shaped host API: one 16 MiB segment
    split into 2 x 8 MiB fragments, encoded, then each of the 3 fragments erased and rebuilt;
    bit-exact vs the C oracle (and the C oracle's threaded single-segment ops agree)."""
    from oracle.c_oracle import ptrs
    k, m, F = 2, 1, 8 * MiB
    seg = np.empty(k * F, np.uint8)
    corc.orc_fill_synthetic(seg.ctypes.data, k * F, 1, 0, 0xCE550001)
    enc = cess.New(k, m)
    shards = enc.Split(seg)
    enc.Encode(shards)
    want = c_encode(corc, k, m, shards[:k])
    assert np.array_equal(shards[2], want[0])
    for e in range(3):
        sh = [s.copy() for s in shards]
        sh[e] = None
        enc.Reconstruct(sh)
        assert all(np.array_equal(a, b) for a, b in zip(sh, shards)), e
    cpu = [shards[0].copy(), shards[1].copy(), np.zeros(F, np.uint8)]
    corc.orc_segment_ops(k, m, ptrs(cpu), F, 4, 1)
    assert all(np.array_equal(a, b) for a, b in zip(cpu, shards))


def test_codecs_on_threads_are_independent(torch, cess, corc):
    """include/cess_ec.h: distinct codecs are independent. Four host threads (ctypes drops the
    GIL inside the C calls), each with its own codec, code, kernel options, decode-cache capacity
    and HIP stream, run encode + per-segment reconstruct loops at the same time; every result is
    bit-exact against the C oracle."""
    import concurrent.futures as cf
    cases = [(2, 1, 4096 + 16, 0, 4096), (10, 4, 4099, 1, 2), (32, 32, 8192, 0, 3),
             (4, 2, 1000, 2, 1), (10, 4, 4096, 0, 4)]

    def work(case):
        k, m, ln, rt_mode, cap = case
        # the last case destroys and recreates its codec every iteration while the others run:
        # cec_destroy waits for its own launches only (no device-wide synchronisation)
        churn = case is cases[-1]
        n = k + m
        rng = np.random.default_rng(k * 31 + m)
        nseg = 6
        data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
        want = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
        enc = cess.New(k, m)
        enc.set_option(4, rt_mode)
        enc.set_option(6, cap)
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            d_data = torch.from_numpy(data).cuda()
            d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
        for it in range(12):
            if churn and it:
                enc.close()
                enc = cess.New(k, m)
                enc.set_option(4, rt_mode)
                enc.set_option(6, cap)
            enc.EncodeBatch(d_data, d_par, nseg, ln, stream=st)
            st.synchronize()
            if not np.array_equal(d_par.cpu().numpy(), want):
                return (case, it, "encode")
            present = np.ones((nseg, n), np.uint8)
            for s in range(nseg):
                present[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 0
            with torch.cuda.stream(st):
                d_data.mul_(torch.from_numpy(present[:, :k, None]).cuda())
                d_par.mul_(torch.from_numpy(present[:, k:, None]).cuda())
            enc.ReconstructBatch(d_data, d_par, nseg, ln, present, stream=st)
            st.synchronize()
            if not (np.array_equal(d_data.cpu().numpy(), data)
                    and np.array_equal(d_par.cpu().numpy(), want)):
                return (case, it, "reconstruct")
            if churn:  # destroy right behind queued launches, then check what they wrote
                enc.EncodeBatch(d_data, d_par, nseg, ln, stream=st)
                enc.ReconstructBatch(d_data, d_par, nseg, ln, present, stream=st)
                enc.close()
                st.synchronize()
                if not np.array_equal(d_par.cpu().numpy(), want):
                    return (case, it, "destroy behind launches")
                enc = cess.New(k, m)
        enc.close()
        return None

    with cf.ThreadPoolExecutor(len(cases)) as ex:
        bad = [r for r in ex.map(work, cases) if r is not None]
    assert not bad, bad


@pytest.mark.parametrize("k,m,ln", [(32, 32, 4096), (32, 32, 4096 + 3), (10, 4, 2048), (4, 2, 999)])
def test_all_parity_lost_is_reencoded(torch, cess, corc, k, m, ln):
    """The pattern 'every data shard present, every parity shard lost' runs the encode kernels
    (RS(32,32): the FFT) instead of a run-time decode program: one pattern for the batch, and
    mixed into a per-segment batch beside other patterns; bit-exact vs the C oracle, data
    untouched."""
    nseg = 6
    rng = np.random.default_rng(k + ln)
    n = k + m
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    enc = cess.New(k, m)
    allpar = np.array([1] * k + [0] * m, np.uint8)
    d_data = to_dev(torch, data)
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc.ReconstructBatch(d_data, d_par, nseg, ln, allpar)
    torch.cuda.synchronize()
    assert np.array_equal(d_par.cpu().numpy(), par)
    assert np.array_equal(d_data.cpu().numpy(), data)
    present = np.ones((nseg, n), np.uint8)
    for s in range(nseg):
        if s % 2:
            present[s, k:] = 0
        else:
            present[s, rng.choice(n, size=m, replace=False)] = 0
    d_data = to_dev(torch, data * present[:, :k, None])
    d_par = to_dev(torch, par * present[:, k:, None])
    enc.ReconstructBatch(d_data, d_par, nseg, ln, present)
    torch.cuda.synchronize()
    assert np.array_equal(d_data.cpu().numpy(), data)
    assert np.array_equal(d_par.cpu().numpy(), par)


def test_large_verify_scratch_not_retained(torch, cess, corc):
    """Batch-sized scratch (a generic code's recomputed parity) is stream-ordered, not a pool
    block: after a 128 MiB-scratch verify completes, the codec holds no more HBM than before
    (the pool rounds to powers of two and keeps its blocks until the codec dies)."""
    k, m, ln, nseg = 10, 4, 4 << 20, 8
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (2, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(2)])
    d_data = to_dev(torch, np.concatenate([data] * (nseg // 2)))
    d_par = to_dev(torch, np.concatenate([par] * (nseg // 2)))
    enc = cess.New(k, m)
    before = enc.stat(3)
    d_par[5, 3, 17] ^= 1
    ok = enc.VerifyBatch(d_data, d_par, nseg, ln)
    assert list(ok) == [s != 5 for s in range(nseg)]
    torch.cuda.synchronize()
    after = enc.stat(3)
    assert after - before < (16 << 20), (before, after)
    # the audit gather's scratch as well (hash only: the gathered chunks are scratch)
    from cess_amd import audit
    d_hex = torch.empty((nseg * (k + m), 512, 64), dtype=torch.uint8, device="cuda")
    audit.audit_chunks(enc, d_data, d_par, nseg, ln, list(range(0, 1024, 2)), d_hex=d_hex)
    torch.cuda.synchronize()
    assert enc.stat(3) - before < (16 << 20)
    enc.close()


@pytest.mark.parametrize("k,m,ln,nseg", [(2, 1, 1 << 16, 9), (2, 1, 4099, 5), (4, 2, 1000, 7),
                                         (10, 4, 4096, 6), (32, 32, 4096, 5)])
def test_verify_batch(torch, cess, corc, k, m, ln, nseg):
    """cec_verify_batch (klauspost Verify over an HBM batch): every segment whose stored parity
    equals the C oracle's encode passes; one flipped byte anywhere in a segment's parity (or
    data) fails that segment only; the batch itself is not modified."""
    rng = np.random.default_rng(k * 13 + ln)
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    enc = cess.New(k, m)
    d_data, d_par = to_dev(torch, data), to_dev(torch, par)
    assert enc.VerifyBatch(d_data, d_par, nseg, ln).all()
    enc.set_option(1, 1)  # the generic recompute-and-compare path as well
    assert enc.VerifyBatch(d_data, d_par, nseg, ln).all()
    enc.set_option(1, 0)
    bad = {1: ("p", m - 1, ln - 1), nseg - 1: ("d", 0, ln // 2)}
    for s, (which, i, off) in bad.items():
        t = d_par if which == "p" else d_data
        t[s, i, off] ^= 0x5A
    for generic in (0, 1):
        enc.set_option(1, generic)
        ok = enc.VerifyBatch(d_data, d_par, nseg, ln)
        assert list(ok) == [s not in bad for s in range(nseg)], generic
    enc.set_option(1, 0)
    for s, (which, i, off) in bad.items():  # restore: the verify wrote nothing else
        t = d_par if which == "p" else d_data
        t[s, i, off] ^= 0x5A
    assert np.array_equal(d_par.cpu().numpy(), par) and np.array_equal(d_data.cpu().numpy(), data)
