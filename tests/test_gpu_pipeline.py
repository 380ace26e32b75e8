"""The C host pipeline (cec_pipeline_*, pinned multi-buffered H2D / encode / D2H + GPU
SegmentList hashes) driven from C (tests/native/pipeline_e2e.c) and from Python
(cess_amd.pipeline), against the C / Python oracles: every sampled segment's fragments and
hashes, delivery order, zero-padded tails, SegmentCount enforcement, callback errors."""
import hashlib
import json
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu
MiB = 1 << 20


@pytest.fixture(scope="module")
def e2e_exe(tmp_path_factory):
    exe = tmp_path_factory.mktemp("native") / "pipeline_e2e"
    lib, orc = f"{ROOT}/cess_amd", f"{ROOT}/oracle/build"
    subprocess.run(["gcc", "-O2", "-pthread", f"{ROOT}/tests/native/pipeline_e2e.c",
                    f"-I{ROOT}/include", f"-L{lib}", "-lcessec", f"-L{orc}", "-loracle",
                    f"-Wl,-rpath,{lib}:{orc}", "-o", str(exe)], check=True)
    return str(exe)


@pytest.mark.parametrize("args", [
    # k m F nseg batch depth hash window uniq check_every tail
    (2, 1, 1 << 19, 41, 8, 3, 1, 2, 41, 1, 12345),   # CESS shape, hashes, padded tail
    (2, 1, 1 << 19, 41, 8, 2, 0, 0, 41, 1, 1),       # no hashing, depth 2
    (4, 2, 4160, 33, 5, 3, 1, 3, 33, 1, 0),          # F % 64 == 0: prefix-digest segment chain
    (32, 32, 1000, 20, 4, 2, 1, 1, 20, 1, 999),      # F % 64 != 0, window 1, wide code
    (10, 4, 4096, 7, 64, 3, 1, 16, 7, 1, 0),         # one partial batch
    # host / hybrid record hashes (cec_pipeline_run_files with the source's size)
    (2, 1, 1 << 19, 41, 8, 3, 2, 0, 41, 1, 12345),   # host SHA-256, padded tail
    (2, 1, 1 << 19, 41, 8, 3, 3, 2, 41, 1, 12345, -1),  # hybrid, auto tail
    (2, 1, 1 << 19, 41, 8, 3, 3, 2, 41, 1, 12345, 0),   # hybrid, GPU takes every fragment
    (2, 1, 1 << 19, 41, 8, 4, 3, 3, 41, 1, 12345, 2),   # hybrid, last 2 batches on the host
    (4, 2, 4160, 33, 5, 3, 3, 3, 33, 1, 0, 1),       # hybrid, F % 64 == 0, k = 4
    (32, 32, 1000, 20, 4, 2, 3, 1, 20, 1, 999, 1),   # hybrid, F % 64 != 0: GPU parity only
    (10, 4, 4096, 7, 64, 3, 2, 16, 7, 1, 0),         # host, one partial batch
])
def test_pipeline_from_c(e2e_exe, args):
    r = subprocess.run([e2e_exe] + [str(a) for a in args], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["pipeline"] == "ok" and out["bad"] == 0 and out["checked"] == args[3]


@pytest.mark.parametrize("hash_on", ["gpu", "host", "hybrid", "auto"])
def test_pipeline_python_records(orc, hash_on):
    """encode_file_records on every hash placement of the C pipeline (GPU hash queue, host
    SHA-256 threads, hybrid): the oracle's SegmentLists, file hash and fragments, from bytes, a
    numpy array and a memoryview."""
    from cess_amd.pipeline import encode_file_records
    as_array = lambda b: np.frombuffer(b, np.uint8)  # noqa: E731
    for size, seg, k, m, wrap in [(5 * MiB + 7, MiB, 2, 1, bytes),
                                  (3 * MiB, MiB // 2, 4, 2, as_array),
                                  (MiB - 3, MiB // 4, 32, 32, memoryview)]:
        blob = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
        frags = {}
        rec, st = encode_file_records(
            wrap(blob), k, m, seg, batch_segments=2, window=2, hash_on=hash_on,
            on_fragment=lambda s, i, v: frags.__setitem__((s, i), hashlib.sha256(v).hexdigest()))
        want = orc.segment_list(blob, k, m, seg)
        assert [(s.hash, s.fragment_list) for s in rec.segments] == want
        assert rec.file_hash == orc.file_hash(want) and rec.size == size
        assert st.segments == len(want) and st.bytes_in == size
        assert len(frags) == len(want) * (k + m)
        for (s, i), h in frags.items():
            assert h.encode() == want[s][1][i]


def test_records_host_path_limits():
    import cess_amd
    from cess_amd.pipeline import encode_file_records
    for hash_on in ("host", "hybrid"):
        with pytest.raises(cess_amd.ErrTooManySegments):
            encode_file_records(bytes(5 * 8192), 2, 1, 8192, max_segments=4, hash_on=hash_on)
        with pytest.raises(cess_amd.ErrShortData):
            encode_file_records(b"", 2, 1, 8192, hash_on=hash_on)


@pytest.mark.parametrize("hash_on,tail,k,m,seg", [
    ("hybrid", -1, 2, 1, MiB), ("hybrid", 0, 2, 1, MiB), ("hybrid", 2, 2, 1, MiB),
    ("host", -1, 2, 1, MiB), ("gpu", -1, 2, 1, MiB), ("hybrid", 1, 4, 2, MiB // 2),
    ("hybrid", 1, 32, 32, 32 * 1000)])
def test_records_session_many_files(orc, tmp_path, hash_on, tail, k, m, seg):
    """One RecordsSession (one pipeline) for several files in one run: ragged tails, a file
    shorter than a segment, a path among in-memory buffers; records and fragments equal the
    oracle's, on_file in file order; the session then takes another file; an empty file in the
    list is an error (ErrShortData) and the session stays usable."""
    import cess_amd
    from cess_amd.pipeline import RecordsSession
    sizes = [5 * seg + 7, 3 * seg, seg - 3, 9 * seg + 1]
    blobs = [np.random.default_rng(100 + i).integers(0, 256, n, dtype=np.uint8).tobytes()
             for i, n in enumerate(sizes)]
    path = tmp_path / "f3.bin"
    path.write_bytes(blobs[3])
    srcs = blobs[:3] + [str(path)]
    want = [orc.segment_list(b, k, m, seg) for b in blobs]
    seen, frags = [], {}
    with RecordsSession(k, m, seg, hash_on=hash_on, batch_segments=2, window=2,
                        tail_batches=tail) as ses:
        recs, st = ses.encode_many(
            srcs, on_fragment=lambda f, s, i, v: frags.__setitem__(
                (f, s, i), hashlib.sha256(v).hexdigest().encode()),
            on_file=lambda f, r, fst: seen.append((f, fst.segments)))
        assert seen == [(f, len(w)) for f, w in enumerate(want)]
        assert st.segments == sum(len(w) for w in want) and st.bytes_in == sum(sizes)
        for f, (r, w) in enumerate(zip(recs, want)):
            assert [(x.hash, x.fragment_list) for x in r.segments] == w, f
            assert r.file_hash == orc.file_hash(w) and r.size == sizes[f]
            for s, sl in enumerate(w):
                assert [frags[(f, s, i)] for i in range(k + m)] == sl[1]
        r2, _ = ses.encode(blobs[2])
        assert [(x.hash, x.fragment_list) for x in r2.segments] == want[2]
        with pytest.raises(cess_amd.ErrShortData):
            ses.encode_many([blobs[0], b"", blobs[1]])
        r3, _ = ses.encode(blobs[1])
        assert [(x.hash, x.fragment_list) for x in r3.segments] == want[1]


def test_pipeline_segment_limit_and_callback_errors():
    import cess_amd
    from cess_amd.pipeline import Pipeline
    blob = np.zeros(5 * 4096 * 2, np.uint8)
    enc = cess_amd.New(2, 1)
    with Pipeline(enc, 4096, batch_segments=2, window=2, max_segments=4) as p:
        with pytest.raises(cess_amd.ErrTooManySegments):
            p.run(blob)
    with Pipeline(enc, 4096, batch_segments=2, window=2) as p:
        def boom(seg, views):
            if seg == 3:
                raise KeyError("stop")
        with pytest.raises(KeyError):
            p.run(blob, on_fragments=boom)
        st = p.run(blob)  # the pipeline is reusable after an aborted run
        assert st.segments == 5


@pytest.mark.parametrize("hash_on", ["auto", "gpu"])
def test_cli_encode_streams_fragments_and_scale(tmp_path, orc, hash_on):
    import sys
    from cess_amd import records
    from cess_amd.segments import SegmentList
    rng = np.random.default_rng(3)
    blob = rng.integers(0, 256, 3 * MiB + 5, dtype=np.uint8).tobytes()
    src = tmp_path / "f.bin"
    src.write_bytes(blob)
    outdir = tmp_path / "frags"
    r = subprocess.run([sys.executable, "-m", "cess_amd.cli", "encode", str(src), "--out",
                        str(outdir), "--segment-size", str(1 << 20), "--scale",
                        str(tmp_path / "deal.scale"), "--hash-on", hash_on],
                       capture_output=True, text=True, timeout=300, check=True, cwd=ROOT)
    rec = json.loads(r.stdout)
    assert rec["pipeline"]["hash_on"] == ("hybrid" if hash_on == "auto" else "gpu")
    want = orc.segment_list(blob, 2, 1, 1 << 20)
    assert [(s["hash"].encode(), [f.encode() for f in s["fragment_list"]])
            for s in rec["segments"]] == want
    assert rec["check_file_spec"] and rec["needed_space"] == 4 * (1 << 20) * 15 // 10
    files = sorted(p.name for p in outdir.iterdir())
    assert files == sorted({f.decode() for _, fl in want for f in fl})
    for p in outdir.iterdir():
        assert hashlib.sha256(p.read_bytes()).hexdigest() == p.name
    assert (tmp_path / "deal.scale").read_bytes() == records.deal_info(
        [SegmentList(h, fl) for h, fl in want])
    # over SegmentCount segments (16 KiB segments: 1001 of them) -> rejected
    big = tmp_path / "big.bin"
    big.write_bytes(bytes(1001 * 16384))
    r = subprocess.run([sys.executable, "-m", "cess_amd.cli", "encode", str(big),
                        "--segment-size", "16384", "--hash-on", hash_on], capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2 and "SegmentCount" in r.stdout


def test_pipelines_on_threads(orc):
    """The north_star's per-GPU sharding from one host: independent codecs each driving their own
    C pipeline (pinned ring, three streams, GPU hash queue) on their own host thread at the same
    time, here two per GPU; every SegmentList equals the oracle's."""
    import concurrent.futures as cf
    from cess_amd.pipeline import encode_file_records
    jobs = [(4 * MiB + 3, MiB, 2, 1, 11), (3 * MiB + 100, MiB, 2, 1, 12),
            (2 * MiB, MiB // 2, 4, 2, 13), (MiB + 1, 10 * 4096, 10, 4, 14)]

    def run(job):
        size, seg, k, m, seed = job
        blob = np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()
        rec, _ = encode_file_records(blob, k, m, seg, batch_segments=2, window=2)
        return [(s.hash, s.fragment_list) for s in rec.segments] == orc.segment_list(blob, k, m,
                                                                                    seg)

    with cf.ThreadPoolExecutor(len(jobs)) as ex:
        assert all(ex.map(run, jobs))


def test_library_first_then_torch():
    """A fresh process that touches libcessec before torch (the C pipeline path needs no torch)
    and then uses torch on the GPU: one HIP runtime in the process (cess_amd._lib.load)."""
    import sys
    code = ("import numpy as np\n"
            "from cess_amd.pipeline import encode_file_records\n"
            "rec, _ = encode_file_records(bytes(3 * 65536), 2, 1, 65536, batch_segments=2, "
            "window=2)\n"
            "import torch\n"
            "x = torch.ones(4, device='cuda')\n"
            "rec2, _ = encode_file_records(bytes(3 * 65536), 2, 1, 65536, hash_on='host')\n"
            "assert rec2.file_hash == rec.file_hash\n"
            "print('ok', int(x.sum().item()))\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert r.returncode == 0 and "ok 4" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("devices,size,seg,k,m", [([0, 0, 0], 7 * MiB + 5, MiB, 2, 1),
                                                  ([0, 0], 3 * MiB, MiB // 2, 4, 2),
                                                  ([0, 0, 0, 0, 0], 2 * MiB, MiB, 2, 1)])
@pytest.mark.parametrize("hash_on", ["auto", "gpu", "host"])
def test_multi_device_file_records(orc, tmp_path, devices, size, seg, k, m, hash_on):
    """One host process sharding a file's segments over several pipelines (here several on GPU 0,
    as an uploader on an 8-GPU node would use 8 devices): the merged records equal the oracle's,
    from an in-memory buffer and from a path; more devices than segments leaves some idle."""
    from cess_amd.pipeline import encode_file_records_multi
    blob = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    want = orc.segment_list(blob, k, m, seg)
    path = tmp_path / "f.bin"
    path.write_bytes(blob)
    for src in (blob, str(path)):
        rec, stats = encode_file_records_multi(src, devices, k, m, seg, window=2,
                                               hash_on=hash_on)
        assert [(s.hash, s.fragment_list) for s in rec.segments] == want
        assert rec.file_hash == orc.file_hash(want) and rec.size == size
        assert sum(st.segments for st in stats) == len(want)


def test_cli_encode_devices(tmp_path):
    """`cli encode --devices 0,0` (segments sharded over two pipelines) prints the same records
    as the one-device encode."""
    import contextlib
    import io
    from cess_amd import cli
    blob = np.random.default_rng(11).integers(0, 256, 3 * MiB + 7, dtype=np.uint8).tobytes()
    src = tmp_path / "f.bin"
    src.write_bytes(blob)
    outs = []
    for extra in ([], ["--devices", "0,0"]):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            assert cli.main(["encode", str(src), "--segment-size", str(MiB)] + extra) == 0
        outs.append(json.loads(buf.getvalue().strip().splitlines()[-1]))
    assert outs[0]["segments"] == outs[1]["segments"]
    assert outs[0]["file_hash"] == outs[1]["file_hash"]


def _pipeline_cases(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k, m = [(2, 1), (4, 2), (10, 4), (3, 5)][int(rng.integers(4))]
        F = int(rng.choice([4096, 4160, 65536, 1000 * 64]))
        nseg = int(rng.integers(1, 23))
        tail = int(rng.integers(0, k * F))
        out.append((k, m, F, nseg, tail, int(rng.choice([1, 2, 3, 5, 8])),
                    int(rng.choice([2, 3, 4, 6])), int(rng.choice([1, 2, 3, 7])),
                    bool(rng.integers(2)), int(rng.integers(1 << 30))))
    return out


@pytest.mark.parametrize("k,m,F,nseg,tail,batch,depth,window,hashing,seed",
                         _pipeline_cases(16, 505))
def test_pipeline_random_shapes(orc, k, m, F, nseg, tail, batch, depth, window, hashing, seed):
    """Randomized ring shapes (batch size, ring depth deeper or shallower than the device slots,
    hash window) over files with ragged tails: every segment's shards equal the oracle's split +
    encode (zero-padded tail), in segment order, and with hashing every record equals the
    oracle's SegmentList."""
    import cess_amd
    from cess_amd.pipeline import Pipeline
    seg = k * F
    size = max(1, (nseg - 1) * seg + tail)
    blob = np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()
    want = orc.segment_list(blob, k, m, seg) if hashing else None
    rs = orc.ReedSolomon(k, m)
    seen, recs = [], {}

    def frags(s, views):
        padded = np.zeros(seg, np.uint8)
        chunk = np.frombuffer(blob[s * seg:(s + 1) * seg], np.uint8)
        padded[:len(chunk)] = chunk
        shards = rs.split(padded.tobytes())
        shards[k:] = rs.encode(shards[:k])
        assert all(np.array_equal(v, np.asarray(x, np.uint8)) for v, x in zip(views, shards)), s
        seen.append(s)

    enc = cess_amd.New(k, m)
    with Pipeline(enc, F, batch_segments=batch, depth=depth, hash=hashing, window=window) as p:
        st = p.run(blob, on_fragments=frags,
                   on_record=(lambda s, sh, fl: recs.__setitem__(s, (sh, list(fl))))
                   if hashing else None)
    enc.close()
    nsegs = -(-size // seg)
    assert seen == list(range(nsegs)) and st.segments == nsegs
    if hashing:
        assert [recs[s] for s in range(nsegs)] == [(h, list(fl)) for h, fl in want]


@pytest.mark.gpu
def test_host_sha_pool_holds_every_pipelines_threads(orc):
    """Several host-hashing pipelines in one process (one per GPU in encode_file_records_multi)
    each bring their own host_threads: the process-wide host SHA-256 pool grows to their sum
    (cec_host_sha_pool_threads), not to the largest; records stay equal to the oracle's."""
    from cess_amd import _lib
    from cess_amd.pipeline import RecordsSession, encode_file_records_multi
    lib = _lib.load()
    t0 = lib.cec_host_sha_pool_threads()
    seg = 1 << 20
    blob = np.random.default_rng(9).integers(0, 256, 6 * seg + 5, dtype=np.uint8).tobytes()
    want = orc.segment_list(blob, 2, 1, seg)
    with RecordsSession(2, 1, seg, 0, "hybrid", batch_segments=2, window=2,
                        host_threads=t0 + 5) as a, \
            RecordsSession(2, 1, seg, 0, "host", batch_segments=2, host_threads=7) as b:
        assert lib.cec_host_sha_pool_threads() >= t0 + 12
        for ses in (a, b):
            rec, _ = ses.encode(blob)
            assert [(x.hash, x.fragment_list) for x in rec.segments] == want
    rec, _ = encode_file_records_multi(blob, [0, 0], 2, 1, seg, hash_on="hybrid",
                                       hash_threads=4, window=2)
    assert [(x.hash, x.fragment_list) for x in rec.segments] == want


def _sharded_rank(rank, world, port, path, seg, q):
    import os
    import torch.distributed as dist
    from cess_amd.segments import encode_file_sharded
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec = encode_file_sharded(path, rank, world, segment_size=seg, batch_segments=2, window=2)
        q.put((rank, None if rec is None else
               ([(s.hash, s.fragment_list) for s in rec.segments], rec.file_hash, rec.size)))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_encode_file_sharded_multi_process(orc, tmp_path, world):
    """One process per rank (gloo group, every rank on GPU 0 here): each encodes its contiguous
    segment range through its own RecordsSession (hybrid hashes), rank 0 gathers the SegmentLists
    and returns the whole-file record, equal to the oracle's (segments, file hash, size)."""
    import socket
    import torch.multiprocessing as mp
    seg = 1 << 20
    blob = np.random.default_rng(31).integers(0, 256, 7 * seg + 333, dtype=np.uint8).tobytes()
    path = tmp_path / "sharded.bin"
    path.write_bytes(blob)
    want = orc.segment_list(blob, 2, 1, seg)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_rank, args=(r, world, port, str(path), seg, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=150) for _ in procs)
    finally:  # a rank that failed leaves the others in the gather: end them (these PIDs only)
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert all(p.exitcode == 0 for p in procs)
    assert all(res[r] is None for r in range(1, world))
    segs, fh, size = res[0]
    assert segs == want and fh == orc.file_hash(want) and size == len(blob)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,seg", [(2, 1, 1 << 20), (4, 2, 4 * 4096)])
@pytest.mark.parametrize("resume,threads", [("1", 16), (None, 4), ("0", 4)])
def test_hybrid_resume_records(orc, monkeypatch, capfd, k, m, seg, resume, threads):
    """The hybrid resume: the host hashes fragment 0 of each segment and the GPU queue continues
    the segment chain from its state (cec_hashq_add_resume). Forced on (CEC_PIPELINE_RESUME=1),
    on by itself below 12 host threads, and forced off there; records of several ragged files in
    one run, and of one file with every batch on the GPU (tail 0), equal the oracle's."""
    from cess_amd.pipeline import RecordsSession
    if resume is None:
        monkeypatch.delenv("CEC_PIPELINE_RESUME", raising=False)
    else:
        monkeypatch.setenv("CEC_PIPELINE_RESUME", resume)
    monkeypatch.setenv("CEC_PIPELINE_TRACE", "1")  # its line says whether the run resumed
    sizes = [7 * seg + 5, 3 * seg, seg - 1, 11 * seg]
    blobs = [np.random.default_rng(300 + i).integers(0, 256, n, dtype=np.uint8).tobytes()
             for i, n in enumerate(sizes)]
    want = [orc.segment_list(b, k, m, seg) for b in blobs]
    for tail in (-1, 0):
        with RecordsSession(k, m, seg, hash_on="hybrid", batch_segments=2, window=2,
                            tail_batches=tail, host_threads=threads) as ses:
            recs, _ = ses.encode_many(blobs)
            for f, (r, w) in enumerate(zip(recs, want)):
                assert [(x.hash, x.fragment_list) for x in r.segments] == w, (tail, f)
        on = resume == "1" or (resume is None and threads < 12)
        assert f"resume {int(on)};" in capfd.readouterr().err, tail
