"""Breakdown of reading a transaction file into device tensors:
native parse (mmap + tokenise), export into pinned host tensors, H2D copy;
and, for comparison, the raw cost of getting the file's bytes into HBM
(pread by 16 threads into pinned memory, then one H2D copy).
    python benchmarks/read_probe.py PATH
"""
import ctypes as C
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from fastapriori_amd.ops import _native  # noqa: E402
from fastapriori_amd.utils.env import num_threads  # noqa: E402


def raw_read(path, nt):
    size = os.path.getsize(path)
    t0 = time.time()
    buf = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    t1 = time.time()
    mv = memoryview(buf.numpy())
    fd = os.open(path, os.O_RDONLY)
    chunk = 64 << 20

    def rd(off):
        n = min(chunk, size - off)
        got = 0
        while got < n:
            got += os.preadv(fd, [mv[off + got:off + n]], off + got)
        return n

    with ThreadPoolExecutor(nt) as ex:
        list(ex.map(rd, range(0, size, chunk)))
    os.close(fd)
    t2 = time.time()
    d = buf.to("cuda", non_blocking=True)
    torch.cuda.synchronize()
    t3 = time.time()
    print(f"raw: bytes {size} pin_alloc {t1 - t0:.3f} pread {t2 - t1:.3f} ({size / (t2 - t1) / 1e9:.1f} GB/s) "
          f"h2d {t3 - t2:.3f} ({size / (t3 - t2) / 1e9:.1f} GB/s)", flush=True)
    del d, buf


def main():
    path = sys.argv[1]
    lib = _native.host()
    nt = num_threads()
    for rep in range(2):
        err = C.c_int(0)
        t0 = time.time()
        h = lib.fa_parse_file(path.encode(), 0, -1, 0, nt, C.byref(err))
        t1 = time.time()
        info = np.zeros(6, dtype=np.int64)
        lib.fa_txndb_info(h, info.ctypes.data)
        n, nnz = int(info[0]), int(info[1])
        off = torch.empty(n + 1, dtype=torch.int64, pin_memory=True)
        items = torch.empty(nnz, dtype=torch.int32, pin_memory=True)
        t2 = time.time()
        ex = np.zeros(max(int(info[2]), 1), dtype=np.int32)
        lib.fa_txndb_export(h, off.data_ptr(), items.data_ptr(), ex.ctypes.data, nt)
        lib.fa_txndb_free(h)
        t3 = time.time()
        d_off, d_items = off.to("cuda", non_blocking=True), items.to("cuda", non_blocking=True)
        torch.cuda.synchronize()
        t4 = time.time()
        print(f"threads {nt} parse {t1 - t0:.3f} pin_alloc {t2 - t1:.3f} export {t3 - t2:.3f} h2d {t4 - t3:.3f} "
              f"lines {n} nnz {nnz}", flush=True)
        del d_off, d_items, off, items
    for rep in range(2):
        raw_read(path, nt)


if __name__ == "__main__":
    main()
