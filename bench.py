#!/usr/bin/env python3
"""bench.py -- BASELINE.json headline: device-resident bitshuffle+LZ4
encode+decode round trip of 4 GiB int16 (G1 correlated noise, default 8 KiB
blocks) on MI355X, as GiB/s and as a fraction of the HBM roofline.

One step (config 2, the default) = bshuf_compress_lz4_dev of the whole 4 GiB
buffer (fused transpose + LZ4 kernel, offset scan, compaction) +
bshuf_decompress_lz4_dev of the framed stream it produced (parallel
block-index rebuild from the framing -- the encoder's offsets are NOT reused --
then fused LZ4 decode + inverse transpose).  Inputs are generated on the
device before timing; nothing crosses PCIe inside the timed region: the
decoder reads the stream length from the encoder's device result word
(bshuf_decompress_lz4_dev_dlen / _batch_dev_dlen), so a step never waits on
the host between the two calls.

The other BASELINE configs (parity-tested separately, not the headline line):
  --config 1  bshuf_bitshuffle + bshuf_bitunshuffle of the 64 MiB int32 ramp
  --config 3  the round trip on 16 GiB float32 G2 (elem_size 4, auto blocks)
  --config 4  the round trip of 128 independent 32 MiB int16 G1 chunks per
              GPU (seed 12345 + global chunk id) through the batched API
              (one launch per kernel for all 128 streams)

Multi-GPU: `--gpus N` without a torch.distributed environment re-launches
itself under torch.distributed.run with N ranks (before touching the GPU);
each rank round-trips its own shard (seed 12345 + rank, or its own 128 chunks
in config 4) -- blocks and shards are independent, so there is no data-path
collective; RCCL carries only the barrier, the max of the per-rank times and
the sum of bytes.  value = total uncompressed bytes of all ranks / max time.

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident GiB/s bitshuffle+LZ4 encode+decode, 4 GiB int16; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)

# kernels the library ran on the pipelined encode's side stream (launch.h
# kPipeSegs; their profiling names end in "_side"): they run beside the parse,
# so their event times overlap the step's other kernels
def overlapped(name):
    return name.endswith("_side")


CONFIGS = {
    1: dict(gen=0, dtype="int32", gib=1.0 / 16, what="shuffle"),
    2: dict(gen=1, dtype="int16", gib=4.0, what="lz4"),
    3: dict(gen=2, dtype="float32", gib=16.0, what="lz4"),
    4: dict(gen=1, dtype="int16", gib=4.0, what="batch", chunk_mib=32, chunks=128),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--gib", type=float, default=None, help="uncompressed GiB per GPU (override)")
    ap.add_argument("--elem-size", type=int, default=None,
                    help="configs 2/3: read the same synthetic bytes as elements of this many bytes")
    ap.add_argument("--block-size", type=int, default=None,
                    help="configs 2/3: block size in elements (0 = the reference's default)")
    ap.add_argument("--cpu-sample-mib", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="skip per-kernel event timing")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group (RCCL on a GPU) and run the barrier / "
                         "MAX / SUM collectives even at world size 1 (tests the N>1 code path)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------- dist utils
def maybe_spawn(args, argv):
    """`--gpus N` with N > 1 outside torch.distributed: start N ranks under
    torch.distributed.run as a CHILD process (nothing has touched the GPU yet)
    and exit with its status."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)
    sys.exit(subprocess.call(cmd, env=env))


def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if world > 1 or args.force_dist:
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def _dist_on():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def dist_info():
    if not _dist_on():
        return None
    import torch.distributed as dist
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "collectives": "barrier + all_reduce MAX/SUM on device tensors"}


def barrier(world):
    if _dist_on():
        import torch.distributed as dist
        dist.barrier()


def reduce_over_ranks(x, world, device, op):
    if not _dist_on():
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(x, world, device):
    import torch.distributed as dist
    return reduce_over_ranks(x, world, device, dist.ReduceOp.MAX)


def sum_over_ranks(x, world, device):
    import torch.distributed as dist
    return reduce_over_ranks(x, world, device, dist.ReduceOp.SUM)


def timed_loop(step, steps, warmup, world, sync, device):
    """W untimed steps, then exactly K steps bracketed by barrier + sync on
    both sides; returns the MAX over ranks of the elapsed seconds."""
    for _ in range(warmup):
        step()
    sync()
    barrier(world)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier(world)
    t1 = time.perf_counter()
    return max_over_ranks(t1 - t0, world, device)


# ------------------------------------------------------------------ profiling
def prof_collect(lib):
    buf = ctypes.create_string_buffer(1 << 16)  # collect() resets: one call
    lib.bshuf_prof_collect(buf, 1 << 16)
    out = {}
    for line in buf.value.decode().splitlines():
        name, cnt, ms = line.split()
        out[name] = (int(cnt), float(ms))
    return out


def load_pmc_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json, written by tools/pmc_traffic.py),
    or None when no PMC pass has been committed."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        return json.load(open(p))
    except Exception:
        return None


def copy_peak_gbps(dev, nbytes=2 << 30, reps=5):
    """Achievable HBM bandwidth on this box: a device-to-device
    copy of nbytes, timed with events on torch's current stream, read + write
    bytes per second.  Outside the timed region."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        b.copy_(a)
    e.record()
    e.synchronize()
    gbps = 2.0 * nbytes * reps / (s.elapsed_time(e) / 1e3) / 1e9
    del a, b
    return gbps


# ------------------------------------------------------------ parity digests
def load_digests():
    """SHA-256 digests of the REFERENCE's own output at full BASELINE sizes
    and for the element-size / block-size modes (tests/golden/vectors.json
    "full" and "modes", made by tests/golden/make_vectors.py from oracle/_ref,
    the reference C compiled from /root/reference)."""
    p = os.path.join(ROOT, "tests", "golden", "vectors.json")
    v = json.load(open(p))
    return {e["name"]: e for e in v["full"] + v.get("modes", [])}


def mode_digest(digests, gen, E, bsz, nbytes):
    """The reference digest of a --elem-size / --block-size line's exact input
    (G1 int16 bytes, seed 12345, first nbytes framed as E-byte elements)."""
    for d in digests.values():
        if (d["name"].startswith("mode_") and gen == 1 and d["elem_size"] == E
                and d["bs"] == bsz and d["nbytes"] == nbytes):
            return d
    return None


def sha256_dev(t, nbytes=None):
    """SHA-256 of the first nbytes of a device tensor, streamed to the host in
    256 MiB slices (bounded host memory)."""
    import hashlib
    import torch
    u8 = t.reshape(-1).view(torch.uint8)
    nbytes = u8.numel() if nbytes is None else int(nbytes)
    h = hashlib.sha256()
    step = 256 << 20
    host = torch.empty(min(step, max(nbytes, 1)), dtype=torch.uint8, pin_memory=True)
    for off in range(0, nbytes, step):
        n = min(step, nbytes - off)
        host[:n].copy_(u8[off:off + n])
        h.update(memoryview(host[:n].numpy()))
    return h.hexdigest()


def check_digests(pairs, world, device):
    """pairs: [(name, what, got, want)].  Every rank learns whether ANY rank
    saw a mismatch (max over ranks), and then all of them exit non-zero."""
    bad = [(n, w, g, x) for n, w, g, x in pairs if g != x]
    for n, w, g, x in bad:
        sys.stderr.write("bench.py: PARITY FAILED %s %s: got %s want %s\n" % (n, w, g, x))
    if max_over_ranks(1.0 if bad else 0.0, world, device) > 0:
        raise SystemExit(3)
    return sorted({n for n, _, _, _ in pairs})


# ---------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _omp_threads(n):
    """Thread count of the reference's OpenMP team (libgomp is already loaded
    by oracle/_ref/libbshuf_ref.so; omp_set_num_threads acts on that copy)."""
    try:
        ctypes.CDLL("libgomp.so.1").omp_set_num_threads(int(n))
        return True
    except OSError:
        return False


def cpu_baseline(sample_mib, cfg):
    """The reference's own C (oracle/_ref, compiled from the reference sources
    by oracle/Makefile) timed on this host on a bounded sample of the same
    workload: on the job's CPU share (OMP_NUM_THREADS) and on 1 thread.
      config 1: the reference's SCALAR build (BASELINE configs[0] names the
                CPU scalar path) is `value`; its AVX2 build rides along;
      config 4: one reference call per 32 MiB chunk, as a per-chunk caller
                (the HDF5 filter) would make them;
      otherwise the AVX2 + OpenMP build (the haswell wheels).
    Falls back to our scalar CPU port (1 thread) when _ref is absent."""
    import numpy as np
    from oracle import REF_SCALAR_SO, Oracle, Reference, reference_available
    o = Oracle()
    gen = cfg["gen"]
    es = {0: 4, 1: 2, 2: 4}[gen]
    affinity = len(os.sched_getaffinity(0))
    # the box's CPU share: OMP_NUM_THREADS when the environment sets it (the
    # affinity mask may list far more cores than the job may use; 256 OpenMP
    # threads on a 16-core share run ~25x slower than 16)
    share = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    scalar_so = REF_SCALAR_SO
    batch = cfg["what"] == "batch"
    if batch:
        cn = cfg["chunk_mib"] * (1 << 20) // es
        k = max(1, sample_mib // cfg["chunk_mib"])
        chunks = [o.gen_g1(cn, 0, 12345 + i) for i in range(k)]
        a = None
    else:
        n = sample_mib * (1 << 20) // es
        a = o.gen_g1(n, 0, 12345) if gen == 1 else (o.gen_g2(n, 0, 12345) if gen == 2 else o.gen_g0(n))
    if reference_available():
        kind = "reference"
        codec = Reference(scalar_so) if cfg["what"] == "shuffle" and os.path.exists(scalar_so) \
            else Reference()
    else:
        codec, kind = o, "port"

    def prepared(c, arrs):
        """Per array: pre-allocated, pre-faulted buffers (BASELINE.md 3 /
        SURVEY 8(d)) and a closure that makes ONE round trip through the
        library's C-ABI directly (no allocation, no copy in the timed pass)."""
        jobs = []
        for x in arrs:
            flat = np.ascontiguousarray(x).view(np.uint8).reshape(-1)
            size, es = x.size, x.dtype.itemsize
            if cfg["what"] == "shuffle":
                mid = np.ones(flat.size, np.uint8)
                back = np.ones(flat.size, np.uint8)
                args = (flat, mid, back, size, es)

                def run(f=flat, m=mid, b=back, n=size, e=es):
                    r1 = c._bitshuffle(f.ctypes.data, m.ctypes.data, n, e, 0)
                    r2 = c._bitunshuffle(m.ctypes.data, b.ctypes.data, n, e, 0)
                    assert r1 >= 0 and r2 >= 0
            else:
                mid = np.ones(max(c.compress_lz4_bound(size, es, 0), 1), np.uint8)
                back = np.ones(flat.size, np.uint8)
                args = (flat, mid, back, size, es)

                def run(f=flat, m=mid, b=back, n=size, e=es):
                    r1 = c._compress_lz4(f.ctypes.data, m.ctypes.data, n, e, 0)
                    r2 = c._decompress_lz4(m.ctypes.data, b.ctypes.data, n, e, 0)
                    assert r1 > 0 and r2 == r1
            jobs.append((run, args))
        return jobs

    def rate(c, arrs, budget_s):
        jobs = prepared(c, arrs)
        for run, _ in jobs:  # untimed pass: touches every page, checks the round trip
            run()
        assert all(np.array_equal(a_[2], a_[0]) for _, a_ in jobs)
        best, reps, t_all = None, 0, time.perf_counter()
        nbytes = sum(x.nbytes for x in arrs)
        while reps < 5 or (time.perf_counter() - t_all < budget_s and reps < 20):
            t0 = time.perf_counter()
            for run, _ in jobs:
                run()
            t2 = time.perf_counter()
            v = nbytes / (t2 - t0) / GIB
            best = v if best is None else max(best, v)
            reps += 1
        return best, reps

    arrs = chunks if batch else [a]
    res = {"unit": "GiB/s", "kind": kind, "cpu_model": cpu_model(), "affinity_cores": affinity,
           "os_cpu_count": os.cpu_count()}
    what = {"shuffle": "bitshuffle+bitunshuffle", "lz4": "bitshuffle+LZ4 compress + decompress",
            "batch": "bitshuffle+LZ4 compress + decompress, one call per 32 MiB chunk"}[cfg["what"]]
    total_mib = sum(x.nbytes for x in arrs) >> 20
    if kind == "reference":
        _omp_threads(share)
        v_all, reps_all = rate(codec, arrs, 8.0)
        one = arrs[:1] if batch else [a[: max(len(a) // 8, 1 << 16)]]
        _omp_threads(1)
        v_one, reps_one = rate(codec, one, 6.0)
        _omp_threads(share)
        build = "SCALAR build (-mno-sse2 -mno-avx -mno-avx2)" if codec.path == scalar_so \
            else "-march=haswell (AVX2) build"
        res.update(value=round(v_all, 3), cores=share, value_1thread=round(v_one, 3),
                   sample="%d MiB %s (seed 12345) on the job's CPU share (OMP_NUM_THREADS), best of %d; "
                          "%d MiB 1-thread, best of %d; %s round trip, pre-faulted buffers, direct "
                          "C-ABI calls (bshuf_* via ctypes, no allocation or copy timed), reference "
                          "compiled from /root/reference -O3 -fopenmp (setup.py flags), %s; "
                          "%d-thread / 1-thread = %.2fx" % (
                              total_mib, cfg["dtype"], reps_all, sum(x.nbytes for x in one) >> 20,
                              reps_one, what, build, share, v_all / v_one))
        if cfg["what"] == "shuffle" and codec.path == scalar_so:
            avx = Reference()
            _omp_threads(share)
            v_avx, _ = rate(avx, arrs, 4.0)
            res["value_avx2_build"] = round(v_avx, 3)
    else:
        one = arrs[:1] if batch else [a[: min(len(a), 1 << 24)]]
        v_one, reps_one = rate(o, one, 8.0)
        res.update(value=round(v_one, 3), cores=1, value_1thread=round(v_one, 3),
                   sample="%d MiB, scalar oracle port, 1 thread, best of %d" % (
                       sum(x.nbytes for x in one) >> 20, reps_one))
    return res


# ----------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    maybe_spawn(args, argv)
    import torch
    world, rank, local = dist_setup(args)
    import bitshuffle_amd as B
    from bitshuffle_amd import api

    if not B.using_HIP() or not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (MI355X)")
    cfg = CONFIGS[args.config]
    gib = args.gib if args.gib is not None else cfg["gib"]
    dev = torch.device("cuda", local)
    dt = {"int16": torch.int16, "int32": torch.int32, "float32": torch.float32}[cfg["dtype"]]
    es = torch.empty(0, dtype=dt).element_size()
    lib = B.lib

    if cfg["what"] == "batch":
        cn = cfg["chunk_mib"] * (1 << 20) // es
        nchunks = max(1, int(gib * GIB) // (cfg["chunk_mib"] << 20))
        xs = [torch.empty(cn, dtype=dt, device=dev) for _ in range(nchunks)]
        for i, x in enumerate(xs):
            B.synth_fill_dev(x, cfg["gen"], seed=12345 + rank * nchunks + i)
        nbytes = cn * es * nchunks
        outs = [torch.empty(B.compress_lz4_bound(cn, es, 0), dtype=torch.uint8, device=dev)
                for _ in xs]
        ys = [torch.empty_like(x) for x in xs]
        state = {}

        shapes = [x.shape for x in xs]

        def step():
            # stream lengths stay on the device: the decoder reads them there
            _, res = api.compress_lz4_batch_dev(xs, outs=outs, sync=False)
            state["res"] = res
            state["dres"] = api.decompress_lz4_batch_dev(outs, shapes, dt, outs=ys, sync=False,
                                                         lengths=res)[1]

        def lengths():  # after the timed region
            counts = state["res"].cpu().tolist()
            state["counts"] = counts
            state["C"] = sum(counts)

        def check():
            lengths()
            return (state["dres"].cpu().tolist() == state["counts"]
                    and all(torch.equal(x, y) for x, y in zip(xs, ys)))
        workload = ("batch of %d independent %d MiB %s G1 chunks per GPU (seed 12345 + global "
                    "chunk id), default 8 KiB blocks, bshuf_*_lz4_batch_dev: one launch per kernel "
                    "for all chunks, device-resident, decoder rebuilds each chunk's block index"
                    % (nchunks, cfg["chunk_mib"], cfg["dtype"]))
    elif cfg["what"] == "shuffle":
        n = int(gib * GIB) // es
        x = torch.empty(n, dtype=dt, device=dev)
        B.synth_fill_dev(x, cfg["gen"], seed=12345 + rank)
        nbytes = n * es
        s_buf = torch.empty_like(x)
        y = torch.empty_like(x)
        state = {"C": 0}

        def step():
            api.bitshuffle_dev(x, out=s_buf)
            api.bitunshuffle_dev(s_buf, out=y)

        def lengths():
            pass

        def check():
            return torch.equal(x, y)
        workload = ("bshuf_bitshuffle + bshuf_bitunshuffle of a %.3g MiB %s ramp (G0), default "
                    "blocks, device-resident" % (nbytes / (1 << 20), cfg["dtype"]))
    elif args.elem_size or args.block_size:
        # the same synthetic bytes, framed with another element size and/or
        # block size through the C-ABI directly (no torch dtype of E bytes)
        E = args.elem_size or es
        bsz = args.block_size or 0
        n = int(gib * GIB) // E // 8 * 8
        nbytes = n * E
        xs = torch.empty((nbytes + es - 1) // es, dtype=dt, device=dev)
        B.synth_fill_dev(xs, cfg["gen"], first=0, seed=12345 + rank)
        x = xs.view(torch.uint8)[:nbytes]
        bound = int(lib.bshuf_compress_lz4_bound(n, E, bsz))
        if bound > (1 << 62):
            raise SystemExit("bench.py: invalid --block-size %d" % bsz)
        comp = torch.empty(bound, dtype=torch.uint8, device=dev)
        wse = torch.empty(max(int(lib.bshuf_compress_lz4_dev_workspace(n, E, bsz)), 256),
                          dtype=torch.uint8, device=dev)
        wsd = torch.empty(max(int(lib.bshuf_decompress_lz4_dev_workspace(bound, n, E, bsz)), 256),
                          dtype=torch.uint8, device=dev)  # capacity-sized (device-held length)
        res_e = torch.empty(1, dtype=torch.int64, device=dev)
        res_d = torch.empty(1, dtype=torch.int64, device=dev)
        y = torch.empty_like(x)
        state = {}
        vp = ctypes.c_void_p

        def step():
            st = vp(torch.cuda.current_stream().cuda_stream)
            r = lib.bshuf_compress_lz4_dev(vp(x.data_ptr()), vp(comp.data_ptr()), n, E, bsz,
                                           vp(wse.data_ptr()), wse.numel(), vp(res_e.data_ptr()),
                                           None, st)
            if r < 0:
                raise SystemExit("bshuf_compress_lz4_dev: %d" % r)
            # the stream length stays on the device (res_e)
            r = lib.bshuf_decompress_lz4_dev_dlen(vp(comp.data_ptr()), vp(res_e.data_ptr()), bound,
                                                  vp(y.data_ptr()), n, E, bsz, vp(wsd.data_ptr()),
                                                  wsd.numel(), vp(res_d.data_ptr()), None, st)
            if r < 0:
                raise SystemExit("bshuf_decompress_lz4_dev_dlen: %d" % r)

        def lengths():
            state["C"] = int(res_e.item())

        def check():
            lengths()
            return int(res_d.item()) == state["C"] and torch.equal(x, y)
        workload = ("bitshuffle+LZ4 encode+decode round trip, %.3g GiB of %s %s bytes per GPU read as "
                    "%d-byte elements, block size %d elements (%d bytes), device-resident, decoder "
                    "rebuilds the block index" % (
                        gib, cfg["dtype"], "G1" if cfg["gen"] == 1 else "G2", E,
                        bsz or B.default_block_size(E), (bsz or B.default_block_size(E)) * E))
        es = E
    else:
        n = int(gib * GIB) // es // 8 * 8
        x = torch.empty(n, dtype=dt, device=dev)
        B.synth_fill_dev(x, cfg["gen"], first=0, seed=12345 + rank)
        nbytes = n * es
        bound = B.compress_lz4_bound(n, es, 0)
        comp = torch.empty(bound, dtype=torch.uint8, device=dev)
        ws_enc = api.compress_lz4_workspace(n, es, 0, device=dev)
        ws_dec = api.decompress_lz4_workspace(bound, n, es, 0, device=dev)
        res_e = torch.empty(1, dtype=torch.int64, device=dev)
        res_d = torch.empty(1, dtype=torch.int64, device=dev)
        y = torch.empty_like(x)
        state = {}

        def step():
            api.compress_lz4_dev(x, out=comp, workspace=ws_enc, result=res_e, sync=False)
            # the stream length stays on the device: the decoder reads res_e
            api.decompress_lz4_dev(comp, x.shape, x.dtype, out=y, workspace=ws_dec,
                                   result=res_d, sync=False, length=res_e)

        def lengths():
            state["C"] = int(res_e.item())

        def check():
            lengths()
            return int(res_d.item()) == state["C"] and torch.equal(x, y)
        workload = ("bitshuffle+LZ4 encode+decode round trip, %.3g GiB %s %s per GPU, default "
                    "blocks (%d elem), device-resident, decoder rebuilds the block index" % (
                        gib, cfg["dtype"], "G1 correlated noise" if cfg["gen"] == 1
                        else "G2 smooth field", B.default_block_size(es)))

    # parity gate before timing: exact round trip, and on every rank that owns
    # a BASELINE input with a committed reference digest, the input and the
    # framed stream byte-for-byte against the REFERENCE's output (length +
    # SHA-256).  Any mismatch exits non-zero before anything is timed.
    step()
    torch.cuda.synchronize()
    if not check():
        raise SystemExit("round trip parity FAILED on rank %d" % rank)
    digests, pairs = load_digests(), []
    if cfg["what"] == "shuffle" and rank == 0 and gib == cfg["gib"]:
        d = digests["cfg1_g0_i32_64MiB"]
        pairs += [(d["name"], "input_sha256", sha256_dev(x), d["input_sha256"]),
                  (d["name"], "shuffled_sha256", sha256_dev(s_buf), d["shuffled_sha256"])]
    elif cfg["what"] == "lz4" and rank == 0 and gib == cfg["gib"] and not (args.elem_size or args.block_size):
        d = digests["cfg2_g1_i16_4GiB" if args.config == 2 else "cfg3_g2_f32_16GiB"]
        pairs += [(d["name"], "input_sha256", sha256_dev(x), d["input_sha256"]),
                  (d["name"], "compressed_len", state["C"], d["compressed_len"]),
                  (d["name"], "compressed_sha256", sha256_dev(comp, state["C"]),
                   d["compressed_sha256"])]
    elif cfg["what"] == "lz4" and rank == 0 and (args.elem_size or args.block_size):
        d = mode_digest(digests, cfg["gen"], es, args.block_size or 0, nbytes)
        if d is not None:
            pairs += [(d["name"], "input_sha256", sha256_dev(x), d["input_sha256"]),
                      (d["name"], "compressed_len", state["C"], d["compressed_len"]),
                      (d["name"], "compressed_sha256", sha256_dev(comp, state["C"]),
                       d["compressed_sha256"])]
    elif cfg["what"] == "batch" and cfg["chunk_mib"] == 32:
        for i in range(nchunks):
            name = "cfg4_g1_chunk%04d" % (rank * nchunks + i)
            if name in digests:
                d = digests[name]
                c = state["counts"][i]
                pairs += [(name, "compressed_len", c, d["compressed_len"]),
                          (name, "compressed_sha256", sha256_dev(outs[i], c), d["compressed_sha256"])]
    checked = check_digests(pairs, world, dev)
    parity = {"kind": "reference-digest" if checked else "self-round-trip",
              "round_trip_exact": True, "digests_matched": checked,
              "source": "tests/golden/vectors.json (reference C output, SHA-256 + length)"}

    # HIP-event timing: every kernel during the warmup steps (the per-kernel
    # breakdown), then ONLY the dominant kernel during the timed steps (the
    # roofline's average launch) -- each timed launch adds two event records
    # to its stream, ~0.2 ms per config-2 step when every kernel is timed
    kern_all, kern = {}, {}
    warm = args.warmup
    if not args.no_prof:
        lib.bshuf_prof_enable(1)
        prof_collect(lib)  # reset
        if warm > 0:
            for _ in range(warm):
                step()
            torch.cuda.synchronize()
            kern_all = prof_collect(lib)
            # (the hipcub scans' event times include waiting for free LDS)
            dom_name = max((k for k in kern_all if not k.startswith("scan_") and not overlapped(k)),
                           key=lambda k: kern_all[k][1])
            lib.bshuf_prof_only(dom_name.encode())
            warm = 0
    elapsed = timed_loop(step, args.steps, warm, world, torch.cuda.synchronize, dev)
    if not args.no_prof:
        kern = prof_collect(lib)
        lib.bshuf_prof_only(None)
        lib.bshuf_prof_enable(0)
        if not kern_all:  # no warmup: every kernel was timed in the timed steps
            kern_all = kern
    breakdown_steps = float(args.warmup if args.warmup > 0 else args.steps)
    lengths()  # the last step's stream length(s), read back after the timed region
    C = state["C"]
    total_bytes = sum_over_ranks(float(nbytes) * args.steps, world, dev)
    value = total_bytes / elapsed / GIB
    ms_step = elapsed / args.steps * 1e3

    roofline = None
    kernels = {}
    if kern:
        # algorithmic bytes per launch, SURVEY.md 8(d): encode N + C, decode
        # C + N, transposes 2N (scratch / index traffic is not credited)
        alg = {"k_lz4_encode": nbytes + C, "k_lz4_decode": C + nbytes, "k_compact": 2 * C,
               "k_compact_side": 2 * C,
               "k_idx_exits": C, "k_seq_scan": C, "k_bitshuffle": 2 * nbytes,
               "k_bitunshuffle": 2 * nbytes}
        for name, (cnt, ms) in kern_all.items():
            kernels[name] = round(ms / cnt, 4)
        dom = max(kern, key=lambda k: kern[k][1])
        avg_s = kern[dom][1] / kern[dom][0] / 1e3
        # a long call runs its parse / decode as several pipelined launches
        # (launch.h kPipeSegs), each over an equal share of the blocks: the
        # algorithmic bytes per launch are the step's bytes / launches per step
        per_step_launches = kern[dom][0] / float(args.steps)
        alg_launch = alg.get(dom, nbytes + C) / per_step_launches
        ach = alg_launch / avg_s / 1e9
        pmc = load_pmc_traffic()
        # only for the workload the committed PMC passes measured: same data,
        # element size, block size and call size (else the per-launch bytes
        # belong to another kernel configuration)
        wl = pmc.get("_workload") if isinstance(pmc, dict) else None
        same = (isinstance(wl, dict) and cfg["what"] == "lz4" and wl.get("gen") == cfg["gen"]
                and wl.get("elem_size") == es and wl.get("block_size") == (args.block_size or 0)
                and wl.get("bytes_per_call") == nbytes)
        traffic = pmc.get(dom) if same else None
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": traffic,
                    "traffic_source": ("profiles/pmc_traffic.json: rocprofv3 FETCH_SIZE/WRITE_SIZE "
                                       "passes committed for this kernel, not measured in this run"
                                       if traffic else None),
                    "alg_bytes_per_launch": int(round(alg_launch)),
                    "launches_per_step": round(per_step_launches, 3),
                    "avg_launch_ms": round(avg_s * 1e3, 4)}
        try:
            cp = copy_peak_gbps(dev)
            roofline["achievable_copy_GBps"] = round(cp, 1)
            roofline["frac_of_achievable"] = round(ach / cp, 4)
        except Exception as e:  # reported, never fatal for the line
            roofline["achievable_copy_GBps"] = None
            roofline["copy_error"] = repr(e)
    # whole round trip priced as SURVEY.md 8(d): 2(N+C) algorithmic bytes per
    # GPU for the codec, 4N for a transpose round trip
    per_step = 4.0 * nbytes if cfg["what"] == "shuffle" else 2.0 * (nbytes + C)
    rt = per_step * args.steps / elapsed / 1e9
    stage = {"alg_GBps_per_gpu": round(rt, 1), "roofline_frac": round(rt / HBM_PEAK_GBS, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.cpu_sample_mib, cfg)
        except Exception as e:  # reported, never fatal for the GPU line
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        metric = METRIC if args.config == 2 else (
            "device-resident GiB/s, BASELINE config %d (%s); %% HBM roofline" % (
                args.config, {1: "bitshuffle+bitunshuffle 64 MiB int32",
                              3: "bitshuffle+LZ4 encode+decode 16 GiB float32",
                              4: "bitshuffle+LZ4 batch of 32 MiB int16 chunks"}[args.config]))
        line = {
            "metric": metric, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": workload, "baseline_config": args.config,
                       "elem_size": es, "block_size": args.block_size or B.default_block_size(es),
                       "bytes_per_gpu": nbytes, "compressed_bytes_rank0": C,
                       "ratio": round(nbytes / C, 4) if C else None,
                       "parallelism": "shard-per-gpu x%d" % world},
            "roofline": roofline, "round_trip": stage,
            # every kernel's event-timed launches in the warmup steps (the
            # timed steps time only the roofline's kernel); side-stream kernels
            # of the pipelined encode (k_compact, scan_block_offsets) overlap
            # the parse, and an event-timed scan includes its wait for free LDS:
            # they are listed apart and do not add to the step
            "kernels_avg_ms": kernels,
            "kernels_ms_per_step": {k: round(v[1] / breakdown_steps, 4)
                                    for k, v in kern_all.items() if not overlapped(k)},
            "kernels_ms_per_step_overlapped": {k: round(v[1] / breakdown_steps, 4)
                                               for k, v in kern_all.items() if overlapped(k)},
            "kernels_timed_in": "warmup steps" if args.warmup > 0 else "timed steps",
            "parity": parity, "cpu_baseline": cpu, "dist": dist_info(),
        }
        print(json.dumps(line), flush=True)
    if _dist_on():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
