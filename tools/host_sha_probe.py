"""Host SHA-256 forms of libcessec (cec_sha256_host) against hashlib on this machine's cores.

Prints one JSON line per measurement: form, threads, chain bytes, GB/s hashed. No GPU needed
(the library is loaded with ctypes; only host entry points are called).
Usage: python tools/host_sha_probe.py [--threads 1,8,16] [--mib 1024]
"""
import argparse
import concurrent.futures as cf
import ctypes
import hashlib
import json
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {0: "scalar", 1: "ni1", 2: "ni2", 3: "ni4", 4: "x16"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,8,16")
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--probe-only", action="store_true")
    ap.add_argument("--lib", default=os.path.join(ROOT, "cess_amd", "libcessec.so"))
    ap.add_argument("--forms", default="1,2,3,4", help="forms timed through cec_sha256_host")
    a = ap.parse_args()
    lib = ctypes.CDLL(a.lib)
    lib.cec_host_sha_probe.restype = ctypes.c_double
    lib.cec_host_sha_probe.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int]
    lib.cec_sha256_host.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                    ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                    ctypes.c_int]
    cpu = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    for form in range(5):
        for w in (1, 2, 4, 16, 18):
            g = lib.cec_host_sha_probe(form, 4 << 20, w)
            if g > 0:
                print(json.dumps({"probe": NAMES[form], "chains": w, "GBps_one_thread": round(g, 3),
                                  "cpu": cpu}), flush=True)
    if a.probe_only:
        return
    total = a.mib << 20
    buf = np.random.default_rng(1).integers(0, 256, total, dtype=np.uint8)
    for chain in (16 << 20, 8 << 20):
        n = total // chain
        ptrs = (ctypes.c_void_p * n)(*[buf.ctypes.data + i * chain for i in range(n)])
        hexo = np.zeros(64 * n, np.uint8)
        want = None
        for th in [int(x) for x in a.threads.split(",")]:
            # hashlib on th threads
            best = 1e9
            for _ in range(a.reps):
                t0 = time.perf_counter()
                with cf.ThreadPoolExecutor(th) as ex:
                    got = list(ex.map(lambda i: hashlib.sha256(
                        memoryview(buf[i * chain:(i + 1) * chain])).hexdigest(), range(n)))
                best = min(best, time.perf_counter() - t0)
            want = got
            print(json.dumps({"form": "hashlib", "threads": th, "chain_MiB": chain >> 20,
                              "GBps": round(total / best / 1e9, 2)}), flush=True)
            for form in [int(f) for f in a.forms.split(",")]:
                if lib.cec_host_sha_set_form(form):
                    continue
                best = 1e9
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    rc = lib.cec_sha256_host(ptrs, n, chain, hexo.ctypes.data, 0, None, th)
                    best = min(best, time.perf_counter() - t0)
                    assert rc == 0
                ok = [bytes(hexo[64 * i:64 * i + 64]).decode() for i in range(n)] == want
                print(json.dumps({"form": NAMES[form], "threads": th, "chain_MiB": chain >> 20,
                                  "GBps": round(total / best / 1e9, 2), "equal_hashlib": ok}),
                      flush=True)
        lib.cec_host_sha_set_form(-1)


if __name__ == "__main__":
    main()
