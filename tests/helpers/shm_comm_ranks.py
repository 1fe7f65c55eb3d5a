"""Worker for tests/test_shm_comm_cpu.py: one rank of the shared-memory
communicator (csrc/shm_comm.h) in host-only mode (no GPU), driving every
collective on host buffers and checking it against numpy in rank order.

usage: shm_comm_ranks.py RANK WORLD PATH SCENARIO
  SCENARIO ok       - all collectives, all dtypes; prints SHM_OK
  SCENARIO mismatch - rank 1 issues a different count; every rank must fail
  SCENARIO timeout  - rank 1 never arrives; rank 0 must time out
"""
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (loads the HIP runtime the extension links)

from mpi_tensorflow_amd.ops import native

F32, BF16, I64 = 7, 9, 4
SUM, MAX = 0, 2


def data(rank, n, dtype, salt=0):
    rs = np.random.RandomState(1000 * rank + 17 * salt + 3)
    if dtype == I64:
        return rs.randint(-1000, 1000, size=n).astype(np.int64)
    x = (rs.randn(n) * 3.0).astype(np.float32)
    if dtype == BF16:
        return (x.view(np.uint32) >> 16).astype(np.uint16)
    return x


def bf2f(u):
    return (u.astype(np.uint32) << 16).view(np.float32)


def f2bf(f):
    u = f.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def ref_reduce(parts, dtype, op):
    if dtype == BF16:
        acc = bf2f(parts[0]).copy()
        for p in parts[1:]:
            acc = np.maximum(acc, bf2f(p)) if op == MAX else (acc + bf2f(p)).astype(np.float32)
        return f2bf(acc)
    acc = parts[0].copy()
    for p in parts[1:]:
        acc = np.maximum(acc, p) if op == MAX else acc + p
    return acc


def addr(a):
    return a.__array_interface__["data"][0]


def main():
    rank, world, path, scen = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    C = native()
    S = C.ShmComm
    timeout = 2.0 if scen != "ok" else 30.0
    cap = 1 << 20
    if rank == 0:
        c = S(path, True, world, 0, cap, timeout, False)
        open(path + ".ready", "w").close()
    else:
        t0 = time.time()
        while not os.path.exists(path + ".ready"):
            if time.time() - t0 > 30:
                raise SystemExit("rank 0 never created the segment")
            time.sleep(0.01)
        c = S(path, False, world, rank, cap, timeout, False)
    if scen == "timeout":
        if rank == 1:
            time.sleep(timeout + 2.0)
            return
        x = data(rank, 100, F32)
        t0 = time.time()
        try:
            c.run_host(S.AR, addr(x), addr(x), 100, F32, SUM, 0)
        except RuntimeError as e:
            dt = time.time() - t0
            assert "did not arrive" in str(e), e
            assert c.async_error() == 6 and dt < timeout + 1.5, (c.async_error(), dt)
            print(f"SHM_TIMEOUT_OK rank={rank} after {dt:.2f}s", flush=True)
            return
        raise SystemExit("the collective completed without its peer")
    if scen == "mismatch":
        n = 100 if rank != 1 else 101
        x = data(rank, n, F32)
        try:
            c.run_host(S.AR, addr(x), addr(x), n, F32, SUM, 0)
        except RuntimeError as e:
            assert "differs" in str(e) or "aborted" in str(e), e
            assert c.async_error() in (5, 6), c.async_error()
            print(f"SHM_MISMATCH_OK rank={rank}: {e}", flush=True)
            return
        raise SystemExit("a mismatched collective was not detected")
    # scen == "ok": every collective, in the same order on every rank
    for dtype in (F32, BF16, I64):
        for op in (SUM, MAX):
            n = 1000 + 37 * dtype  # not a multiple of the chunk size
            parts = [data(r, n, dtype, op) for r in range(world)]
            x = parts[rank].copy()
            c.run_host(S.AR, addr(x), addr(x), n, dtype, op, 0)
            want = ref_reduce(parts, dtype, op)
            assert np.array_equal(x.view(np.uint8), want.view(np.uint8)), ("all_reduce", dtype, op)
            # reduce_scatter: each rank gets its slice of the reduction
            m = 257
            parts = [data(r, m * world, dtype, 7 + op) for r in range(world)]
            out = np.zeros(m, parts[0].dtype)
            c.run_host(S.RS, addr(parts[rank]), addr(out), m, dtype, op, 0)
            want = ref_reduce(parts, dtype, op)[rank * m:(rank + 1) * m]
            assert np.array_equal(out.view(np.uint8), want.view(np.uint8)), ("reduce_scatter", dtype)
        # all_gather
        parts = [data(r, 333, dtype, 11) for r in range(world)]
        out = np.zeros(333 * world, parts[0].dtype)
        c.run_host(S.AG, addr(parts[rank]), addr(out), 333, dtype, SUM, 0)
        assert np.array_equal(out, np.concatenate(parts)), ("all_gather", dtype)
        # broadcast from the last rank, in place
        root = world - 1
        x = data(rank, 500, dtype, 13)
        c.run_host(S.BC, addr(x), addr(x), 500, dtype, SUM, root)
        assert np.array_equal(x, data(root, 500, dtype, 13)), ("broadcast", dtype)
        # reduce to rank 1: non-roots keep their buffer
        parts = [data(r, 700, dtype, 17) for r in range(world)]
        x = parts[rank].copy()
        c.run_host(S.RD, addr(x), addr(x), 700, dtype, SUM, 1)
        want = ref_reduce(parts, dtype, SUM) if rank == 1 else parts[rank]
        assert np.array_equal(x.view(np.uint8), want.view(np.uint8)), ("reduce", dtype)
    big = np.ones((cap // 4) + 1, np.float32)
    try:
        c.run_host(S.AR, addr(big), addr(big), big.size, F32, SUM, 0)
        raise SystemExit("capacity not enforced")
    except RuntimeError as e:
        assert "capacity" in str(e), e
    assert c.async_error() == 0 and c.completed == 3 * 2 * 2 + 3 * 3, c.completed
    print(f"SHM_OK rank={rank} world={world} ops={c.completed}", flush=True)


if __name__ == "__main__":
    main()
