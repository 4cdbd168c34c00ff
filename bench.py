#!/usr/bin/env python3
"""bench.py -- BASELINE.json headline: device-resident bitshuffle+LZ4
encode+decode round trip of 4 GiB int16 (G1 correlated noise, default 8 KiB
blocks) on MI355X, as GiB/s and as a fraction of the HBM roofline.

One step = bshuf_compress_lz4_dev of the whole 4 GiB buffer (fused transpose +
LZ4 kernel, offset scan, compaction) + bshuf_decompress_lz4_dev of the framed
stream it produced (parallel block-index rebuild from the framing -- the
encoder's offsets are NOT reused -- then fused LZ4 decode + inverse transpose).
Inputs are generated on the device before timing; nothing crosses PCIe inside
the timed region except the 8-byte compressed length the decoder needs.

Multi-GPU (launched by torch.distributed.run): every rank round-trips its own
4 GiB shard (seed 12345 + rank) -- blocks and shards are independent, so there
is no data-path collective; RCCL is used only for the barrier and the max of
the per-rank times.  value = total uncompressed bytes of all ranks / max time.

Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident GiB/s bitshuffle+LZ4 encode+decode, 4 GiB int16; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GIB = float(1 << 30)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--gib", type=float, default=4.0, help="uncompressed GiB per GPU")
    ap.add_argument("--cpu-sample-mib", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true", help="skip per-kernel event timing")
    return ap.parse_args(argv)


# ----------------------------------------------------------------- dist utils
def dist_setup(args):
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world, device):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, device):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


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


# ---------------------------------------------------------------- CPU baseline
def cpu_baseline(sample_mib):
    """The reference's own C (oracle/_ref: AVX2 + OpenMP build from the
    reference sources) timed on this host, on a bounded sample of the same
    workload.  Falls back to our scalar CPU port when _ref is absent."""
    import numpy as np
    from oracle import Oracle, Reference, reference_available
    o = Oracle()
    n = sample_mib * (1 << 20) // 2
    a = o.gen_g1(n, 0, 12345)
    if reference_available():
        codec, kind = Reference(), "reference"
        cores = int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count())))
    else:
        codec, kind, cores = o, "port", 1
        a = a[: min(n, 1 << 24)]
    best = None
    t_all = time.perf_counter()
    reps = 0
    while reps < 3 or (time.perf_counter() - t_all < 8.0 and reps < 50):
        t0 = time.perf_counter()
        c = codec.compress_lz4(a)
        t1 = time.perf_counter()
        d = codec.decompress_lz4(c, a.shape, a.dtype)
        t2 = time.perf_counter()
        if reps == 0:
            assert np.array_equal(d, a)
        v = a.nbytes / (t2 - t0) / GIB
        best = v if best is None else max(best, v)
        reps += 1
    return {"value": round(best, 3), "unit": "GiB/s", "cores": cores, "kind": kind,
            "sample": "%d MiB int16 G1 (seed 12345), bitshuffle+LZ4 compress + decompress "
                      "round trip through the C-ABI, best of %d reps; %s" % (
                          a.nbytes >> 20, reps,
                          "reference C from /root/reference compiled -O3 -march=haswell "
                          "-fopenmp (setup.py flags)" if kind == "reference"
                          else "scalar oracle port, 1 thread")}


# ----------------------------------------------------------------------- main
def main(argv=None):
    args = parse_args(argv)
    import torch
    world, rank, local = dist_setup(args)
    import bitshuffle_amd as B
    from bitshuffle_amd import api

    if not B.using_HIP() or not torch.cuda.is_available():
        raise SystemExit("bench.py needs a HIP device (MI355X)")
    dev = torch.device("cuda", local)
    nbytes = int(args.gib * GIB) // 16 * 16
    n = nbytes // 2
    x = torch.empty(n, dtype=torch.int16, device=dev)
    B.synth_fill_dev(x, 1, first=0, seed=12345 + rank)
    bound = B.compress_lz4_bound(n, 2, 0)
    comp = torch.empty(bound, dtype=torch.uint8, device=dev)
    ws_enc = api.compress_lz4_workspace(n, 2, 0, device=dev)
    ws_dec = api.decompress_lz4_workspace(bound, n, 2, 0, device=dev)
    res_e = torch.empty(1, dtype=torch.int64, device=dev)
    res_d = torch.empty(1, dtype=torch.int64, device=dev)
    y = torch.empty_like(x)
    clen = [0]

    def step():
        api.compress_lz4_dev(x, out=comp, workspace=ws_enc, result=res_e, sync=False)
        c = int(res_e.item())  # the decoder needs the stream length on the host
        clen[0] = c
        api.decompress_lz4_dev(comp[:c], x.shape, x.dtype, out=y, workspace=ws_dec, result=res_d,
                               sync=False)

    # parity gate before timing: exact round trip + consumed == produced
    step()
    torch.cuda.synchronize()
    if int(res_d.item()) != clen[0] or not torch.equal(x, y):
        raise SystemExit("round trip parity FAILED on rank %d" % rank)

    lib = B.lib
    if not args.no_prof:
        lib.bshuf_prof_enable(1)
        prof_collect(lib)  # reset
    elapsed = timed_loop(step, args.steps, args.warmup, world, torch.cuda.synchronize, dev)
    kern = {}
    if not args.no_prof:
        kern = prof_collect(lib)
        lib.bshuf_prof_enable(0)
    # the warmup steps are also in the event log: count only per-launch averages
    C = clen[0]
    total_bytes = sum_over_ranks(float(nbytes) * args.steps, world, dev)
    value = total_bytes / elapsed / GIB
    ms_step = elapsed / args.steps * 1e3

    roofline = None
    kernels = {}
    if kern:
        alg = {"k_lz4_encode": nbytes + C, "k_lz4_decode": C + nbytes, "k_compact": C,
               "k_idx_exits": C, "k_bitshuffle": 2 * nbytes, "k_bitunshuffle": 2 * nbytes}
        for name, (cnt, ms) in kern.items():
            kernels[name] = round(ms / cnt, 4)
        dom = max(kern, key=lambda k: kern[k][1])
        avg_s = kern[dom][1] / kern[dom][0] / 1e3
        ach = alg.get(dom, nbytes + C) / avg_s / 1e9
        pmc = load_pmc_traffic()
        traffic = pmc.get(dom) if isinstance(pmc, dict) else None
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "alg_bytes_per_launch": alg.get(dom, nbytes + C),
                    "avg_launch_ms": round(avg_s * 1e3, 4)}
    # whole round trip priced as SURVEY.md 8(d): 2(N+C) algorithmic bytes per GPU
    rt = 2.0 * (nbytes + C) * args.steps / elapsed / 1e9
    stage = {"alg_GBps_per_gpu": round(rt, 1), "roofline_frac": round(rt / HBM_PEAK_GBS, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.cpu_sample_mib)
        except Exception as e:  # reported, never fatal for the GPU line
            cpu = {"value": None, "error": repr(e)}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "bitshuffle+LZ4 encode+decode round trip, %.3g GiB int16 G1 "
                                   "correlated noise per GPU, default 8 KiB blocks (4096 elem), "
                                   "device-resident, decoder rebuilds the block index" % args.gib,
                       "elem_size": 2, "block_size": 4096, "bytes_per_gpu": nbytes,
                       "compressed_bytes_rank0": C, "ratio": round(nbytes / max(C, 1), 4),
                       "parallelism": "shard-per-gpu x%d" % world},
            "roofline": roofline, "round_trip": stage, "kernels_avg_ms": kernels,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
