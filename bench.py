#!/usr/bin/env python3
"""Benchmark: device-resident Leopard-RS encode + decode through the C ABI.

Metric (BASELINE.json): device-resident encode+decode GB/s of input bytes
(original_count * buffer_bytes per object, the reference's own formula,
tests/benchmark.cpp:521-524).

Headline workload (configs[1]): 128 originals + 128 recovery pieces of 65536
bytes, GF(2^8).  One *step* = one pass over OBJECTS independent objects
(default 64, a storage node's stripes): each is encoded and then decoded with
every original lost (the benchmark's worst case, rebuilt from the 128 recovery
pieces).  Default mode "batch": the objects go out in launches of
--launch-objects (default 64: the whole step, one encode and one decode
launch) through the leo_amd_encode_batch / leo_amd_decode_batch extension,
consecutive launch pairs alternating over 2 streams; the line records mode and
objects per launch (16 / 32 / 64 objects per launch measured 1127-1140 /
1151-1170 / 1181-1193 GB/s, profiles/r05_v2/headline_launch_sweep.txt).
`modes` also carries the drop-in comparable figures through the reference
C ABI: "calls_in_flight" (leo_encode + leo_decode per object, 3 streams in
flight, async device pointers) and "serial" (one stream, each call waiting for
the previous: a plain drop-in caller).  The steps cycle through enough buffer
sets to exceed 512 MiB (> 2x the 256 MiB Infinity Cache), so every step reads
HBM.  Every rank codes its own objects (64-byte column blocks and objects never
interact; no collective): "scaling": "weak", value = input bytes of all ranks /
max-over-ranks time.

configs[4] (`sharded_object`): ONE 32768+32768 x 64 KiB object (2 GiB of
originals, GF(2^16)) column-sharded over the N ranks -- rank g runs
leo_amd_encode_slice / leo_amd_decode_slice on its B/N columns of every piece,
which it alone allocates (pieces of B/N bytes holding those columns' bytes)
-- timed with a barrier and max over ranks ("strong" scaling: the object is
fixed as N grows).  With N > 1, rank 0 also times the whole object alone on
its GPU in the same run, so the line carries the 1-GPU time of that object.

Roofline: the kernel of the headline's timed region (batch mode: the
encode-batch and decode-batch launches, k_ff8_bs_slab<1> / <2>), timed inside
that region with HIP events recorded right before and after every launch on
its stream.  Consecutive launch pairs on 2 streams overlap (a launch's ramp-up
runs under the previous one's drain), so the launch time is the GPU time per
launch over the region, (last post-launch event - first pre-launch event) /
launches ("launch_us"); each launch's own pre->post span (= rocprofv3's kernel
duration, which counts the overlapped time twice) is reported beside it.
achieved = algorithmic bytes per launch (objects x ((K + R) * B encode,
(K_surv + lost) * B decode)) / launch_us, against the 8 TB/s
HBM3E peak.  traffic = HBM bytes per
launch from the committed rocprofv3 PMC pass (tools/pmc_traffic.py), when
present for this workload.  roofline.single_call carries the same figures for
one leo_encode / leo_decode call (the plain drop-in caller's kernel).

cpu_baseline: the reference library compiled from its sources
(oracle/_ref/libleopard_ref.so, AVX2 + OpenMP) on this host: the headline
workload on 1 core (its FF8 path has no OpenMP), plus the GF(2^16) shapes at 1
and all allowed threads, warm and cold single-call (the reference's own
methodology, tests/benchmark.cpp:420-429, 471-480), and the CPU model.
Falls back to our scalar oracle port if the reference build is absent.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VP = ctypes.c_void_p

# Benchmarks.md:8-27 (reference, "few year old laptop", AVX2, B = 2560 except 128+128 at 64000),
# input MB/s (encode, decode): the breadth shapes
BREADTH = [  # (K, R, B, losses, ref enc MB/s, ref dec MB/s)
    (100, 10, 2560, 10, 5333.33, 1695.36),
    (100, 20, 2560, 20, 3878.79, 833.876),
    (128, 128, 64000, 128, 1964.98, 600.542),
    (1000, 200, 2560, 200, 1942.34, 367.109),
    (1000, 1000, 2560, 1000, 1038.54, 365.876),
    (32768, 32768, 2560, 32768, 471.209, 164.957),
    (32768, 2048, 2560, 2048, 1359.71, 169.359),
]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--R", type=int, default=128)
    ap.add_argument("--bytes", type=int, default=65536)
    ap.add_argument("--objects", type=int, default=64, help="independent objects per step")
    ap.add_argument("--launch-objects", type=int, default=64,
                    help="batch mode: objects per leo_amd_*_batch launch (a step is objects / launch-objects launches)")
    ap.add_argument("--sets", type=int, default=0, help="buffer sets rotated (0 = enough for >512 MiB)")
    ap.add_argument("--streams", type=int, default=3,
                    help="per-call mode: object o of a step runs on HIP stream o %% S")
    ap.add_argument("--mode", choices=("batch", "calls"), default="batch",
                    help="batch: a step is one leo_amd_encode_batch + one leo_amd_decode_batch over its objects "
                         "(one launch each); calls: one leo_encode + leo_decode per object, S streams in flight")
    ap.add_argument("--batch-streams", type=int, default=2,
                    help="batch mode: consecutive steps alternate over this many streams")
    ap.add_argument("--sharded-steps", type=int, default=0, help="steps of the configs[4] object (0 = min(steps, 10))")
    ap.add_argument("--no-sharded", action="store_true", help="skip the configs[4] sharded object")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--no-secondary", action="store_true", help="skip 1000+200, B=64000 and the breadth shapes")
    ap.add_argument("--no-host", action="store_true", help="skip the host-memory (PCIe-inclusive) rate")
    ap.add_argument("--stub", action="store_true",
                    help="launcher test (tests/test_cpu_bench_launcher.py): ranks rendezvous, barrier and take the "
                         "max over ranks of a stand-in time, with no GPU work")
    return ap.parse_args()


def launch_ranks(n):
    """`bench.py --gpus N` run without a launcher (no WORLD_SIZE): start N rank
    processes of this script, one per GPU, and return the first non-zero exit
    code.  They are fresh interpreters started from this one before it makes
    any GPU call (it never makes one), with RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set as torch.distributed.run would set them; rank 0 prints the
    line.  A rank that fails ends the others (they would wait at a barrier)."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def stub_rank(world, rank):
    """--stub: the launcher's control plane alone (gloo rendezvous, barrier,
    max over ranks), for the CPU test of launch_ranks."""
    import torch.distributed as dist
    from leopard_amd.sharding import max_over_ranks
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    el = max_over_ranks(0.25 * (rank + 1))
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, {"rank": rank, "pid": os.getpid()})
        dist.destroy_process_group()
    else:
        ranks = [{"rank": 0, "pid": os.getpid()}]
    if rank == 0:
        print(json.dumps({"stub": True, "world": world, "max_over_ranks": el, "ranks": ranks}), flush=True)


def hash_fill_cuda(torch, seed, pieces, nbytes, device, full_bytes=None, col0=0):
    """Synthetic piece bytes on the device: a 32-bit counter hash of the global
    byte index (same bytes as tests/oracle_lib.hash_bytes).  With full_bytes:
    columns [col0, col0 + nbytes) of pieces of full_bytes bytes (a column
    shard holds the same bytes as those columns of the whole object)."""
    out = torch.empty((pieces, nbytes), dtype=torch.uint8, device=device)
    flat = out.view(-1)
    step = 1 << 26
    M = 0xFFFFFFFF
    for s in range(0, flat.numel(), step):
        e = min(flat.numel(), s + step)
        g = torch.arange(s, e, dtype=torch.int64, device=device)
        if full_bytes is not None:
            g = (g // nbytes) * full_bytes + col0 + g % nbytes
        x = (g * 2654435761 + seed * 0x632BE5AB) & M
        x = x ^ (x >> 16)
        x = (x * 0x85EBCA6B) & M
        x = x ^ (x >> 13)
        x = (x * 0xC2B2AE35) & M
        x = x ^ (x >> 16)
        flat[s:e] = (x & 0xFF).to(torch.uint8)
    return out


def ptrs(t, rows=None, lost=()):
    n = t.shape[0] if rows is None else rows
    lost = set(lost)
    return (VP * n)(*[None if i in lost else t[i].data_ptr() for i in range(n)])


class Sets:
    """Pre-built pointer arrays (ctypes) for rotating buffer sets."""

    def __init__(self, leo, torch, k, r, nbytes, nsets, device):
        self.k, self.r, self.nbytes = k, r, nbytes
        self.enc_wc = leo.leo_encode_work_count(k, r)
        self.dec_wc = leo.leo_decode_work_count(k, r)
        self.orig, self.enc_work, self.dec_work = [], [], []
        self.p_orig, self.p_encw, self.p_null, self.p_rec, self.p_decw = [], [], [], [], []
        for s in range(nsets):
            o = hash_fill_cuda(torch, 7 + s, k, nbytes, device)
            ew = torch.zeros((self.enc_wc, nbytes), dtype=torch.uint8, device=device)
            dw = torch.zeros((self.dec_wc, nbytes), dtype=torch.uint8, device=device)
            self.orig.append(o)
            self.enc_work.append(ew)
            self.dec_work.append(dw)
            self.p_orig.append(ptrs(o))
            self.p_encw.append(ptrs(ew))
            self.p_null.append((VP * k)())  # every original lost
            self.p_rec.append(ptrs(ew, r))
            self.p_decw.append(ptrs(dw))
        self.n = nsets


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # before anything touches a GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:
        return stub_rank(world, rank)
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")  # control plane only (barrier, max-time); no data-path collective
    # one process per GPU (device = local rank); more ranks than GPUs (a
    # functional rehearsal on a smaller box) share devices round-robin, and the
    # line says so (n_gpus = distinct devices, world = ranks)
    ndev = max(1, torch.cuda.device_count())
    gpu = local % ndev
    if ndev >= int(os.environ.get("LOCAL_WORLD_SIZE", world)):
        assert gpu == local, "each rank owns a distinct device"
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)
    placement = [(os.uname().nodename, gpu)]
    if world > 1:
        placement = [None] * world
        dist.all_gather_object(placement, (os.uname().nodename, gpu))
    n_devices = len(set(placement))

    import leopard_amd as leo
    from leopard_amd.sharding import max_over_ranks
    assert leo.leo_init() == 0, leo.last_error()
    stream = torch.cuda.current_stream(device)
    leo.set_stream(stream.cuda_stream)
    leo.set_async(True)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    head = headline(args, leo, torch, device, barrier, world, max_over_ranks)

    sharded = None
    if not args.no_sharded:
        sharded = configs4_sharded(args, leo, torch, device, barrier, rank, world, max_over_ranks, n_devices)

    secondary = breadth = host = cpu = None
    if rank == 0 and not args.no_secondary:
        secondary = [run_shape(leo, torch, device, *c, n=10) for c in
                     ((1000, 200, 65536, 200), (1000, 200, 64000, 200), (128, 128, 64000, 128),
                      (128, 128, 65536, 16))]
        breadth = [dict(run_shape(leo, torch, device, k, r, b, loss, n=5),
                        reference_MBps={"encode": re, "decode": rd, "source": "Benchmarks.md:8-27"})
                   for k, r, b, loss, re, rd in BREADTH]
        secondary.append(dict(ff16_batch(leo, torch, device), kind="ff16_batch"))
    if rank == 0 and not args.no_host:
        host = host_e2e(leo, args.K, args.R, args.bytes)
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.K, args.R, args.bytes, args.cpu_seconds)

    if rank == 0:
        k, r, nbytes = args.K, args.R, args.bytes
        batch = args.mode == "batch"
        kern1 = kernels_for(k, r, nbytes, k)
        traffic = pmc_traffic(head["dominant"][0], k, r, nbytes, head["launch_objects"] if batch else 1,
                              kernels="k_ff8_bs_slab" if batch else kern1[head["dominant"][0]], loss=k)
        kind, algo, t_kernel = head["dominant"]
        achieved = algo / t_kernel / 1e9
        s_kind, s_algo, s_t = head["single_dominant"]
        s_traffic = pmc_traffic(s_kind, k, r, nbytes, 1, kernels=kern1[s_kind], loss=k)
        kname = ("k_ff8_bs_slab<1> / <2>: %d-object encode-batch / decode-batch launches (bit-sliced tile; "
                 "dense encode form / full-loss decode form)" % head["launch_objects"]) if batch else kind
        out = {
            "metric": "device-resident encode+decode GB/s (input bytes/s) at 128+128 and 32768+32768 pieces",
            "value": head["value"],
            "unit": "GB/s",
            "n_gpus": n_devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-hash bytes on device)",
            # the secondary configs' times / roofline fractions and the PCIe-inclusive host rate as
            # top-level scalars (a record that keeps the head of the line or drops nested objects
            # still has them); the same figures sit in `roofline`, `host_e2e` and `secondary`
            **config_fracs(secondary, sharded, world),
            **({"breadth_100x10_decode_us": breadth[0]["decode_us"]} if breadth else {}),
            "host_e2e_GBps": host["value"] if host else None,
            "host_encode_GBps": host["encode_GBps"] if host else None,
            "config": {"workload": f"configs[1]: {k}+{r} x {nbytes} B pieces, GF(2^8); step = {args.objects} objects "
                                   f"per rank, each encoded then decoded with all {k} originals lost, "
                                   + (f"batched encode + decode launches of {head['launch_objects']} objects, "
                                      f"consecutive launch pairs on {args.batch_streams} streams"
                                      if args.mode == "batch" else f"{head['streams']} objects in flight")
                                   + f"; {head['sets']} rotating buffer sets"
                                   + (f"; plus configs[4] (sharded_object): one 32768+32768 x 65536 B object "
                                      f"column-sharded over {world} rank(s) on {n_devices} GPU(s)" if sharded else ""),
                       "original_count": k, "recovery_count": r, "buffer_bytes": nbytes, "losses": k,
                       "objects_per_step": args.objects, "objects_per_launch": head["launch_objects"], "mode": args.mode,
                       "field": "FF8" if leo.leo_decode_work_count(k, r) <= 256 else "FF16",
                       "sharding": "objects per rank (headline); 64-byte column blocks per rank (sharded_object); "
                                   "no collective",
                       # scalars the driver's record keeps (it drops nested objects): ranks and their devices,
                       # and the PCIe-inclusive host rate (never `value`)
                       "world": world, "devices": ",".join(f"{h}:{g}" for h, g in placement),
                       "shared_devices": n_devices < world,
                       "host_e2e_GBps": host["value"] if host else None,
                       "host_encode_GBps": host["encode_GBps"] if host else None,
                       "host_decode_GBps": host["decode_GBps"] if host else None,
                       "host_registered_GBps": host["registered"]["value"] if host else None},
            "modes": head["modes"],
            "encode_GBps": round(k * nbytes / head["t_enc"] / 1e9, 3),
            "decode_GBps": round(k * nbytes / head["t_dec"] / 1e9, 3),
            "encode_us": round(head["t_enc"] * 1e6, 3),
            "decode_us": round(head["t_dec"] * 1e6, 3),
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic.get("bytes"), "traffic_source": traffic.get("source"),
                         "algorithmic_bytes_per_launch": algo, "launch_us": round(t_kernel * 1e6, 3),
                         "launch_time": ("busy: GPU time per launch over the timed region, (last post-launch "
                                         "event - first pre-launch event) / launches; span: one launch's own "
                                         "pre->post event interval, the rocprofv3 kernel-trace duration, which "
                                         "counts the time it overlaps the neighbouring launch on the other "
                                         "stream" if batch else "back-to-back single calls behind a spin kernel"),
                         # busy is this rank's wall GPU time per launch: where ranks share a device the
                         # other ranks' launches run inside it, so the fraction is not the kernel's own
                         **({"shared_device": True,
                             "shared_device_note": "ranks share a device: launch_us holds the other ranks' "
                                                   "launches too; achieved / frac understate the kernel"}
                            if n_devices < world else {}),
                         **({"launch_span_encode_us": round(head["span_enc"] * 1e6, 3),
                             "launch_span_decode_us": round(head["span_dec"] * 1e6, 3)} if batch else {}),
                         # per-config fractions as scalars (the driver's record keeps scalars only)
                         "single_call_us": round(s_t * 1e6, 3),
                         "single_call_frac": round(s_algo / s_t / 1e9 / HBM_PEAK_GBPS, 4),
                         **config_fracs(secondary, sharded, world),
                         "single_call": {"kernel": s_kind, "launch_us": round(s_t * 1e6, 3),
                                         "achieved": round(s_algo / s_t / 1e9, 2),
                                         "frac": round(s_algo / s_t / 1e9 / HBM_PEAK_GBPS, 4),
                                         "traffic": s_traffic.get("bytes"), "traffic_source": s_traffic.get("source"),
                                         "algorithmic_bytes_per_launch": s_algo}},
            "cpu_baseline": cpu,
            "sharded_object": sharded,
            "host_e2e": host,
            "secondary": secondary,
            "breadth": breadth,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def config_fracs(secondary, sharded, world):
    """Roofline fractions and times of configs[2] (1000+200 x 64 KiB, 200
    random losses) and configs[3] (32768+32768 x 64 KiB, full loss; whole
    object only at N = 1), flat."""
    out = {}
    if secondary:
        c2 = secondary[0]
        out.update({"configs2_encode_us": c2["encode_us"], "configs2_decode_us": c2["decode_us"],
                    "configs2_encode_frac": c2["roofline"]["encode"]["frac"],
                    "configs2_decode_frac": c2["roofline"]["decode"]["frac"]})
        if len(secondary) > 3:
            c1p = secondary[3]  # 128+128 x 64 KiB, 16 random losses (partial-loss decoder)
            out["configs1_16loss_decode_us"] = c1p["decode_us"]
        for sec in secondary:
            if sec.get("kind") == "ff16_batch":
                out["ff16_batch_speedup_encode"] = sec["speedup_encode"]
                out["ff16_batch_speedup_decode"] = sec["speedup_decode"]
    if sharded and world == 1:
        pc = sharded["per_call"]
        out.update({"configs3_encode_ms": pc["encode"]["ms"], "configs3_decode_ms": pc["decode"]["ms"],
                    "configs3_encode_frac": pc["encode"]["frac"], "configs3_decode_frac": pc["decode"]["frac"]})
    if sharded:
        out["configs4_GBps"] = sharded["value"]
        out["configs4_roundtrip_ok"] = sharded["roundtrip_ok"]
    return out


def headline(args, leo, torch, device, barrier, world, max_over_ranks):
    lib = leo.lib
    stream = torch.cuda.current_stream(device)
    k, r, nbytes = args.K, args.R, args.bytes
    per_set = (k + leo.leo_encode_work_count(k, r) + leo.leo_decode_work_count(k, r)) * nbytes
    lobj = max(1, min(args.launch_objects, args.objects))
    nsets = args.sets or max(16, args.objects, lobj * max(1, args.batch_streams), -(-(512 << 20) // per_set))
    sets = Sets(leo, torch, k, r, nbytes, nsets, device)
    torch.cuda.synchronize()

    def enc(i):
        return lib.leo_encode(nbytes, k, r, sets.enc_wc, sets.p_orig[i], sets.p_encw[i])

    def dec(i):
        return lib.leo_decode(nbytes, k, r, sets.dec_wc, sets.p_null[i], sets.p_rec[i], sets.p_decw[i])

    # correctness gate before timing: a decode must reproduce the originals
    assert enc(0) == 0 and dec(0) == 0, leo.last_error()
    torch.cuda.synchronize()
    assert torch.equal(sets.dec_work[0][:k], sets.orig[0]), "decode mismatch"
    for i in range(sets.n):
        assert enc(i) == 0
    torch.cuda.synchronize()

    # Per-call mode: object o of a step (encode of buffer set i, then the
    # decode of its recovery pieces) runs on stream o % S; calls on one stream
    # stay ordered and concurrent objects never share buffers.
    nstreams = max(1, args.streams)
    streams = [torch.cuda.Stream(device) for _ in range(nstreams)]

    def run_calls(nsteps, ns):
        for s in range(nsteps):
            for o in range(args.objects):
                i = (s * args.objects + o) % sets.n
                leo.set_stream(streams[o % ns].cuda_stream)
                if enc(i) != 0 or dec(i) != 0:
                    raise RuntimeError(leo.last_error())

    # Batch mode: step s covers buffer sets (s * objects + o) % n, o < objects,
    # in launches of lobj objects: one leo_amd_encode_batch and one
    # leo_amd_decode_batch (one kernel launch each) per group, consecutive groups
    # alternating over --batch-streams streams (their buffer sets differ, so one
    # group's encode overlaps the previous group's decode tail); the pointer
    # arrays are built once per distinct group.
    PP = ctypes.POINTER(VP)
    nbatches = sets.n // lobj if sets.n % lobj == 0 else sets.n
    batches = []
    for bi in range(nbatches):
        ids = [(bi * lobj + o) % sets.n for o in range(lobj)]
        mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
        batches.append((mk([sets.p_orig[i] for i in ids]), mk([sets.p_encw[i] for i in ids]),
                        mk([sets.p_null[i] for i in ids]), mk([sets.p_rec[i] for i in ids]),
                        mk([sets.p_decw[i] for i in ids])))
    bstreams = [stream] + [torch.cuda.Stream(device) for _ in range(max(1, args.batch_streams) - 1)]
    groups = -(-args.objects // lobj)

    # ev (timed region only): four events per launch pair, on the pair's stream
    # right before and after each of its two launches.
    def run_batches(nsteps, _ns, ev=None):
        for s in range(nsteps):
            for g in range(groups):
                j = s * groups + g
                cnt = min(lobj, args.objects - g * lobj)
                st = bstreams[j % len(bstreams)]
                leo.set_stream(st.cuda_stream)
                bo, bw, bn, br, bd = batches[(s * args.objects // lobj + g) % nbatches]
                if ev is not None:
                    ev[4 * j].record(st)
                rc = lib.leo_amd_encode_batch(cnt, nbytes, k, r, sets.enc_wc, bo, bw)
                if ev is not None:
                    ev[4 * j + 1].record(st)
                    ev[4 * j + 2].record(st)
                rc = rc or lib.leo_amd_decode_batch(cnt, nbytes, k, r, sets.dec_wc, bn, br, bd)
                if ev is not None:
                    ev[4 * j + 3].record(st)
                if rc != 0:
                    raise RuntimeError(leo.last_error())

    def timed(run, ns, ev=None):
        run(args.warmup, ns)
        barrier()
        t0 = time.perf_counter()
        if ev is None:
            run(args.steps, ns)
        else:
            run(args.steps, ns, ev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        el = max_over_ranks(t1 - t0)
        if world > 1:
            barrier()
        return el

    # correctness gate of the batch path before timing it
    for i in range(sets.n):
        sets.dec_work[i].zero_()
    run_batches(1, 1)
    torch.cuda.synchronize()
    for o in range(args.objects):
        i = o % sets.n
        assert torch.equal(sets.dec_work[i][:k], sets.orig[i]), "batch decode mismatch"
    elapsed_calls = timed(run_calls, nstreams)
    elapsed_serial = timed(run_calls, 1)
    # the headline's launch events: allocated before the timed region, read after it
    batch_ev = [torch.cuda.Event(enable_timing=True) for _ in range(4 * args.steps * groups)]
    elapsed_batch = timed(run_batches, 1, batch_ev)
    elapsed = elapsed_batch if args.mode == "batch" else elapsed_calls
    leo.set_stream(stream.cuda_stream)

    # Per-launch kernel duration with HIP events on the launch stream: a spin
    # kernel holds the stream while the host enqueues n back-to-back calls (one
    # kernel each on the FF8 path) between one event pair, so the pair holds
    # only GPU time; back-to-back kernels start as the previous one ends
    # (rocprofv3 trace: median gap 0), so time / n is the mean launch duration.
    def time_calls(fn, n=100):
        for j in range(10):
            fn(j % sets.n)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(50_000_000)
        e0.record(stream)
        for j in range(n):
            fn(j % sets.n)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / n

    t_enc = time_calls(enc)
    t_dec = time_calls(dec)
    algo_enc = (k + r) * nbytes
    algo_dec = (r + k) * nbytes  # R surviving pieces read + K lost originals written (full loss)
    dominant = ("decode", algo_dec, t_dec) if t_dec >= t_enc else ("encode", algo_enc, t_enc)

    # The batch mode's kernels, timed inside the headline's timed region itself
    # from the events recorded right before and after every encode-batch and
    # decode-batch launch on its stream (one kernel per launch on this path):
    #  - span: a launch's own pre->post interval (what rocprofv3's kernel trace
    #    reports as its duration).  With --batch-streams 2 consecutive launches
    #    overlap (one launch's ramp-up runs under the previous one's drain), so a
    #    span counts the overlapped time in both launches;
    #  - busy: GPU time per launch = (last post - first pre) / launches; equal to
    #    span + gap with one stream, and the time each launch adds to the GPU's
    #    busy time when they overlap (any idle GPU time counts against it).
    # tb_* (the roofline's launch time) is busy; spans are reported beside it.
    npairs = args.steps * groups
    span_enc = sum(batch_ev[4 * j].elapsed_time(batch_ev[4 * j + 1]) for j in range(npairs)) / npairs / 1e3
    span_dec = sum(batch_ev[4 * j + 2].elapsed_time(batch_ev[4 * j + 3]) for j in range(npairs)) / npairs / 1e3
    last = max(batch_ev[0].elapsed_time(batch_ev[4 * j + 3]) for j in range(max(0, npairs - 4), npairs))
    busy = last / (2 * npairs) / 1e3
    tb_enc = tb_dec = busy
    del batch_ev
    algo_batch = args.objects * (k + r) * nbytes / groups  # mean objects per launch x bytes per object
    batch_dominant = (("decode", algo_batch, tb_dec) if tb_dec >= tb_enc else ("encode", algo_batch, tb_enc))
    if args.mode == "batch":
        dominant, single_dominant = batch_dominant, dominant
    else:
        single_dominant = dominant
    in_step = k * nbytes * args.objects

    def rate(el, note):
        return {"value": round(world * in_step * args.steps / el / 1e9, 3),
                "ms_per_step": round(el / args.steps * 1e3, 4), "note": note}

    res = {"value": round(world * in_step * args.steps / elapsed / 1e9, 3),
           "ms_per_step": round(elapsed / args.steps * 1e3, 4),
           "modes": {
               "batch": rate(elapsed_batch, f"leo_amd_encode_batch + leo_amd_decode_batch per {lobj} objects "
                                            f"(one launch each), {groups} launch pairs per step, consecutive pairs "
                                            f"on {len(bstreams)} stream(s)"),
               "calls_in_flight": rate(elapsed_calls, f"one leo_encode + leo_decode per object, {nstreams} objects "
                                                      f"in flight on {nstreams} streams"),
               "serial": rate(elapsed_serial, "one leo_encode + leo_decode per object on one stream: each call "
                                              "waits for the previous (a plain drop-in caller)")},
           "t_enc": t_enc, "t_dec": t_dec, "tb_enc": tb_enc, "tb_dec": tb_dec,
           "span_enc": span_enc, "span_dec": span_dec, "dominant": dominant,
           "single_dominant": single_dominant, "sets": sets.n, "streams": nstreams, "launch_objects": lobj}
    del sets
    torch.cuda.empty_cache()
    return res


def configs4_sharded(args, leo, torch, device, barrier, rank, world, max_over_ranks, n_devices=None):
    """BASELINE configs[4]: one 32768+32768 x 64 KiB object, column-sharded over
    the ranks (leopard_amd.sharding -> leo_amd_encode_slice / decode_slice; the
    codec being sharded is LeopardFF16.cpp:1397-1467, 1652-1775).  Each rank
    allocates only its own column shard of every piece (its columns of the
    object's bytes, as B/N-byte pieces: memory and placement as in a real
    N-way split) and codes it with the slice calls at offset 0."""
    from leopard_amd.sharding import shard_for_rank
    lib = leo.lib
    k = r = 32768
    b = 65536
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    off, size = shard_for_rank(b, rank, world)
    stream = torch.cuda.current_stream(device)
    leo.set_stream(stream.cuda_stream)

    def shard(width, col0):  # pieces of `width` bytes = columns [col0, col0 + width) of the object
        data = hash_fill_cuda(torch, 7, k, width, device, full_bytes=b, col0=col0)
        work = torch.empty((wc, width), dtype=torch.uint8, device=device)
        dwork = torch.empty((dwc, width), dtype=torch.uint8, device=device)
        return data, work, dwork, (ptrs(data), ptrs(work), ptrs(work, r), ptrs(dwork))

    pn = (VP * k)()  # every original lost

    def step(width, p):
        po, pw, pr, pd = p
        if lib.leo_amd_encode_slice(width, 0, width, k, r, wc, po, pw) != 0:
            raise RuntimeError(leo.last_error())
        if lib.leo_amd_decode_slice(width, 0, width, k, r, dwc, pn, pr, pd) != 0:
            raise RuntimeError(leo.last_error())

    data, work, dwork, pp = shard(size, off)
    step(size, pp)
    torch.cuda.synchronize()
    ok = bool(torch.equal(dwork[:k], data))
    if world > 1:  # every rank's columns round-trip
        ok = max_over_ranks(0.0 if ok else 1.0) == 0.0
    nsteps = args.sharded_steps or max(1, min(args.steps, 10))
    step(size, pp)
    barrier()
    t0 = time.perf_counter()
    for _ in range(nsteps):
        step(size, pp)
    torch.cuda.synchronize()
    el_local = time.perf_counter() - t0
    el = max_over_ranks(el_local)
    n1_ms = None
    if world > 1:  # the same object on one GPU (rank 0 alone, whole pieces) for the strong-scaling ratio
        barrier()
        if rank == 0:
            full = shard(b, 0)
            step(b, full[3])
            torch.cuda.synchronize()
            a = time.perf_counter()
            for _ in range(max(1, nsteps // 2)):
                step(b, full[3])
            torch.cuda.synchronize()
            n1_ms = (time.perf_counter() - a) / max(1, nsteps // 2) * 1e3
            del full
            torch.cuda.empty_cache()
        barrier()
    ms = el / nsteps * 1e3
    ndev = n_devices or world  # distinct GPUs under the ranks (ranks may share one)
    algo = 2 * (k + r) * b  # encode (K + R) * B + full-loss decode (R + K) * B, whole object
    res = {"workload": f"configs[4]: one {k}+{r} x {b} B object (GF(2^16), encode + full-loss decode), "
                       f"column-sharded over {world} rank(s) on {ndev} GPU(s): "
                       f"{b // world if b % world == 0 else size} B of every "
                       f"piece per rank, allocated per rank as pieces of that width (its columns of the "
                       f"object's bytes), via leo_amd_encode_slice / leo_amd_decode_slice",
           "value": round(k * b * nsteps / el / 1e9, 3), "unit": "GB/s", "scaling": "strong",
           "n_gpus": ndev, "world": world, "ms_per_step": round(ms, 3), "steps": nsteps, "roundtrip_ok": ok,
           "roofline": {"bound": "hbm", "achieved_per_gpu": round(algo / ndev / (ms / 1e3) / 1e9, 2),
                        "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(algo / ndev / (ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                        "algorithmic_bytes_per_step": algo}}
    # configs[3] per call on this rank's columns: encode alone, decode alone (HIP events on the
    # call stream), with the kernels the library runs and the committed PMC traffic (full width)
    def timed(fn, reps=3):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / reps

    po, pw, pr, pd = pp

    def enc():
        if lib.leo_amd_encode_slice(size, 0, size, k, r, wc, po, pw) != 0:
            raise RuntimeError(leo.last_error())

    def dec():
        if lib.leo_amd_decode_slice(size, 0, size, k, r, dwc, pn, pr, pd) != 0:
            raise RuntimeError(leo.last_error())

    kern = kernels_for(k, r, size, k)
    per = {}
    for kind, fn in (("encode", enc), ("decode", dec)):
        cms = timed(fn)
        algo1 = (k + r) * size
        t = pmc_traffic(kind, k, r, b, kernels=kern[kind], loss=k) if size == b else {}
        per[kind] = {"ms": round(cms, 3), "kernel": kern[kind], "achieved": round(algo1 / cms / 1e6, 2),
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(algo1 / cms / 1e6 / HBM_PEAK_GBPS, 4),
                     "algorithmic_bytes": algo1, "traffic": t.get("bytes"), "traffic_source": t.get("source")}
    res["per_call"] = per
    # every rank's own step time and slice-kernel times (where strong scaling is lost:
    # a slow rank, or slices whose kernels do not shrink with the columns)
    mine = {"rank": rank, "columns": [off, size], "ms_per_step": round(el_local / nsteps * 1e3, 3),
            "encode_ms": per["encode"]["ms"], "decode_ms": per["decode"]["ms"]}
    if world > 1:
        import torch.distributed as dist
        allr = [None] * world
        dist.all_gather_object(allr, mine)
        res["per_rank"] = allr
    else:
        res["per_rank"] = [mine]
    if n1_ms is not None:
        res["one_gpu_ms_per_step"] = round(n1_ms, 3)
        res["speedup_vs_one_gpu"] = round(n1_ms / ms, 3)
    del data, work, dwork
    torch.cuda.empty_cache()
    return res


def kernels_for(k, r, nbytes, loss):
    """The kernels the library runs for one encode / one decode of this shape
    (mirrors the dispatch in leopard_amd.cpp; names as rocprofv3 lists them)."""
    m = 1 << (r - 1).bit_length()
    n = 1 << (m + k - 1).bit_length()
    if n <= 256:
        enc = "k_ff8_enc"
        if loss == k == r == m:
            dec = "k_ff8_enc (inverse form)"
        elif 2 * m == n:
            dec = "k_ff8_dec_half" if loss == k else "k_ff8_dec_split"
        else:
            dec = "k_ff8_dec"
        return {"encode": enc, "decode": dec}
    narrow = nbytes <= 256 << 10
    enc = ("k_enc16n" if narrow and m in (128, 256) else
           "k_enc_fused" if m <= 256 and not (m == 256 and k > m and nbytes < 512 << 10) else "k_enc_lo + k_enc_hi + k_enc_fin")
    nout = ((m + k - 1) >> 8) - (m >> 8) + 1  # 256-position tiles holding originals
    dec = (("k_dec16n_one" if nbytes >= 60 << 10 and nout <= 4 else "k_dec16n_lo + k_dec16n_fin") if narrow and n <= 2048 else
           "k_el16 (new pattern) + k_dec_lo + k_dec_hi%s + k_dec_fin" % ("_half" if loss == k and 2 * m == n else ""))
    return {"encode": enc, "decode": dec}


def run_shape(leo, torch, device, k, r, nbytes, loss, n=3):
    """One (K, R, B) shape: encode, then decode with `loss` originals lost (the
    benchmark's ShuffleDeck16 pattern, tests/benchmark.cpp:440-467).  Per-call
    GPU time with HIP events on the call stream: a spin kernel holds the stream
    while the host enqueues n back-to-back calls over buffer sets rotated so
    that their total exceeds the 256 MiB MALL (no cache-warm re-reads)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as ol  # the reference benchmark's PCG + ShuffleDeck16 loss pattern
    lib = leo.lib
    ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    per_set = (k + ewc + dwc) * nbytes
    nsets = max(1, min(16, -(-(512 << 20) // per_set)))
    lo, lr = ol.benchmark_losses(k, r, loss, seed=2, trial=0)
    sets = []
    for j in range(nsets):
        o = hash_fill_cuda(torch, 7 + j, k, nbytes, device)
        ew = torch.empty((ewc, nbytes), dtype=torch.uint8, device=device)
        dw = torch.empty((dwc, nbytes), dtype=torch.uint8, device=device)
        sets.append((o, ew, dw, ptrs(o), ptrs(ew), ptrs(dw), ptrs(o, lost=lo), ptrs(ew, r, lost=lr)))
    s = torch.cuda.current_stream(device)
    leo.set_stream(s.cuda_stream)

    def t(fn):
        for j in range(nsets):
            assert fn(j) == 0, leo.last_error()
        s.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        z = torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        a.record(s)
        for j in range(n):
            assert fn(j % nsets) == 0, leo.last_error()
        z.record(s)
        z.synchronize()
        return a.elapsed_time(z) / 1e3 / n

    te = t(lambda j: lib.leo_encode(nbytes, k, r, ewc, sets[j][3], sets[j][4]))
    td = t(lambda j: lib.leo_decode(nbytes, k, r, dwc, sets[j][6], sets[j][7], sets[j][5]))
    idx = torch.tensor(lo, device=device)
    ok = all(bool(torch.equal(st[2].index_select(0, idx), st[0].index_select(0, idx))) for st in sets)
    inb = k * nbytes
    field = "GF(2^8)" if dwc <= 256 else "GF(2^16)"
    kern = kernels_for(k, r, nbytes, loss)

    def roof(kind, us, algo):  # roofline of the call's kernels, PMC traffic when committed for this shape
        t = pmc_traffic(kind, k, r, nbytes, kernels=kern[kind], loss=loss)
        return {"bound": "hbm", "kernel": kern.get(kind) if isinstance(kern, dict) else None,
                "achieved": round(algo / us / 1e3, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(algo / us / 1e3 / HBM_PEAK_GBPS, 4), "algorithmic_bytes": algo,
                "traffic": t.get("bytes"), "traffic_source": t.get("source")}
    res = {"workload": f"{k}+{r} x {nbytes} B, {field}, {loss} originals lost", "encode_GBps": round(inb / te / 1e9, 3),
           "decode_GBps": round(inb / td / 1e9, 3), "encode_decode_GBps": round(inb / (te + td) / 1e9, 3),
           "encode_us": round(te * 1e6, 2), "decode_us": round(td * 1e6, 2), "roundtrip_ok": ok,
           "buffer_sets": nsets, "kernels": kern,
           "roofline_frac": {"encode": round((k + r) * nbytes / te / 1e9 / HBM_PEAK_GBPS, 4),
                             "decode": round((k + loss) * nbytes / td / 1e9 / HBM_PEAK_GBPS, 4)},
           "roofline": {"encode": roof("encode", te * 1e6, (k + r) * nbytes),
                        "decode": roof("decode", td * 1e6, (k + loss) * nbytes)}}
    del sets
    torch.cuda.empty_cache()
    return res


def ff16_batch(leo, torch, device, k=1000, r=200, nbytes=2560, objects=16, loss=200, n=10):
    """GF(2^16) objects of the breadth shape 1000+200 x 2560 B (Benchmarks.md:
    17-27): `objects` single leo_encode / leo_decode calls against one
    leo_amd_encode_batch + one leo_amd_decode_batch over the same objects (one
    grid per kernel), GPU time per object (HIP events behind a spin kernel)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as ol
    lib = leo.lib
    ewc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    lo, lr = ol.benchmark_losses(k, r, loss, seed=2, trial=0)
    data = [hash_fill_cuda(torch, 11 + o, k, nbytes, device) for o in range(objects)]
    ew = [torch.zeros((ewc, nbytes), dtype=torch.uint8, device=device) for _ in range(objects)]
    dw = [torch.zeros((dwc, nbytes), dtype=torch.uint8, device=device) for _ in range(objects)]
    po = [ptrs(d) for d in data]
    pe = [ptrs(e) for e in ew]
    pn = [ptrs(d, lost=lo) for d in data]
    pr = [ptrs(e, r, lost=lr) for e in ew]
    pd = [ptrs(d) for d in dw]
    PP = ctypes.POINTER(VP)
    mk = lambda arrs: (PP * len(arrs))(*[ctypes.cast(a, PP) for a in arrs])  # noqa: E731
    bo, be, bn, br, bd = mk(po), mk(pe), mk(pn), mk(pr), mk(pd)
    s = torch.cuda.current_stream(device)
    leo.set_stream(s.cuda_stream)

    def single_enc():
        for o in range(objects):
            assert lib.leo_encode(nbytes, k, r, ewc, po[o], pe[o]) == 0, leo.last_error()

    def single_dec():
        for o in range(objects):
            assert lib.leo_decode(nbytes, k, r, dwc, pn[o], pr[o], pd[o]) == 0, leo.last_error()

    def batch_enc():
        assert lib.leo_amd_encode_batch(objects, nbytes, k, r, ewc, bo, be) == 0, leo.last_error()

    def batch_dec():
        assert lib.leo_amd_decode_batch(objects, nbytes, k, r, dwc, bn, br, bd) == 0, leo.last_error()

    def t(fn):
        fn()
        s.synchronize()
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        a.record(s)
        for _ in range(n):
            fn()
        z.record(s)
        z.synchronize()
        return a.elapsed_time(z) / 1e3 / n / objects * 1e6  # us per object
    res = {"workload": f"{objects} objects of {k}+{r} x {nbytes} B (GF(2^16), {loss} originals lost each)",
           "single_encode_us_per_object": round(t(single_enc), 2), "single_decode_us_per_object": round(t(single_dec), 2),
           "batch_encode_us_per_object": round(t(batch_enc), 2), "batch_decode_us_per_object": round(t(batch_dec), 2)}
    for d in dw:
        d.zero_()
    batch_dec()
    idx = torch.tensor(lo, device=device)
    res["roundtrip_ok"] = all(bool(torch.equal(dw[o].index_select(0, idx), data[o].index_select(0, idx)))
                              for o in range(objects))
    res["speedup_encode"] = round(res["single_encode_us_per_object"] / res["batch_encode_us_per_object"], 2)
    res["speedup_decode"] = round(res["single_decode_us_per_object"] / res["batch_decode_us_per_object"], 2)
    del data, ew, dw
    torch.cuda.empty_cache()
    return res


def host_e2e(leo, k, r, nbytes, steps=20):
    """PCIe-inclusive rates (never `value`): the same encode + full-loss decode
    step through the C ABI on caller-owned host buffers (the reference's
    contract), (a) plain pageable buffers, staged by the library through its
    pinned ring, and (b) the same buffers registered with leo_amd_register_host,
    which the kernels read and write in place over PCIe."""
    plain = host_e2e_run(leo, k, r, nbytes, steps, register=False)
    reg = host_e2e_run(leo, k, r, nbytes, steps, register=True)
    out = dict(plain)
    out["registered"] = reg
    return out


def host_e2e_run(leo, k, r, nbytes, steps, register):
    import numpy as np
    data = np.frombuffer(np.random.default_rng(7).bytes(k * nbytes), dtype=np.uint8).reshape(k, nbytes).copy()
    wc, dwc = leo.leo_encode_work_count(k, r), leo.leo_decode_work_count(k, r)
    work = np.zeros((wc, nbytes), dtype=np.uint8)
    dwork = np.zeros((dwc, nbytes), dtype=np.uint8)
    po = [data[i].ctypes.data for i in range(k)]
    pe = [work[i].ctypes.data for i in range(wc)]
    pr = [work[i].ctypes.data for i in range(r)]
    pd = [dwork[i].ctypes.data for i in range(dwc)]
    lost = [None] * k
    if register:
        for arr in (data, work, dwork):
            assert leo.register_host(arr.ctypes.data, arr.nbytes) == 0, leo.last_error()

    def step():
        assert leo.leo_encode(nbytes, k, r, wc, po, pe) == 0, leo.last_error()
        assert leo.leo_decode(nbytes, k, r, dwc, lost, pr, pd) == 0, leo.last_error()

    step()
    t0 = time.perf_counter()
    t_enc = 0.0
    for _ in range(steps):
        a = time.perf_counter()
        assert leo.leo_encode(nbytes, k, r, wc, po, pe) == 0, leo.last_error()
        t_enc += time.perf_counter() - a
        assert leo.leo_decode(nbytes, k, r, dwc, lost, pr, pd) == 0, leo.last_error()
    dt = time.perf_counter() - t0
    ok = bool(np.array_equal(dwork[:k], data))
    if register:
        for arr in (data, work, dwork):
            leo.unregister_host(arr.ctypes.data)
    inb = k * nbytes
    how = ("registered host buffers (leo_amd_register_host): kernels read and write them in place over PCIe"
           if register else "pageable numpy buffers (rows of one array): direct SDMA row copies H2D, kernels, D2H per call")
    return {"value": round(inb * steps / dt / 1e9, 3), "unit": "GB/s", "encode_GBps": round(inb * steps / t_enc / 1e9, 3),
            "decode_GBps": round(inb * steps / (dt - t_enc) / 1e9, 3), "roundtrip_ok": ok,
            "sample": f"{steps} steps of {k}+{r} x {nbytes} B encode + full-loss decode, {how}"}


def _profile_order(path):
    """(round, version) of profiles/rNN_vMM/...: newest first when sorted in reverse."""
    import re
    m = re.search(r"r(\d+)_v(\d+)", path)
    return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)


def kernel_bases(names):
    """The kernel base names (template arguments dropped) in a '+'-joined list,
    without the ones a call launches only for a new erasure pattern."""
    import re
    return frozenset(m.group(1) for m in re.finditer(r"(k_[A-Za-z0-9_]+)(?:<[^>]*>)?( \(new pattern\))?", names)
                     if not m.group(2))


def pmc_traffic(role, k, r, nbytes, objects=1, kernels=None, loss=None):
    """HBM bytes per launch of one role ("encode" / "decode") of a workload from
    the newest committed PMC pass (tools/pmc_traffic.py: FETCH_SIZE x 2 +
    WRITE_SIZE, MI355X_MICROARCH.md HBM section; profiles/rNN_vMM ordered by
    round, then version) -- only when the counted kernels are the ones this call
    runs (`kernels`, as kernels_for names them) and, for a decode, the counted
    number of lost originals is this call's (`loss`; a pass without a recorded
    loss ran tools/kbench.py, which loses min(K, R)); else {} (the line then
    says traffic: null)."""
    import glob
    want = kernel_bases(kernels) if kernels else None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_traffic*.json")), key=_profile_order,
                       reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        key = f"{k}+{r}x{nbytes}" + (f"/batch{objects}" if objects > 1 else "")
        e = d.get("workloads", {}).get(key, {}).get(role)
        if not e:
            continue
        if want is not None and kernel_bases(e.get("kernel", "")) != want:
            continue
        if role == "decode" and loss is not None and e.get("loss", min(k, r)) != loss:
            continue
        return {"bytes": e["hbm_bytes_per_launch"], "source": os.path.relpath(path, REPO), "kernel": e.get("kernel")}
    return {}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(k, r, nbytes, seconds):
    """The reference library (or our scalar port) on this host.

    value: the headline workload (128+128 x 64 KiB, encode + full-loss decode)
    on 1 core, warm buffers (the reference's GF(2^8) path is single-threaded).
    detail: cold single calls as tests/benchmark.cpp:420-429, 471-480 time them
    (fresh zero-filled buffers, first touch inside the call, one call), and the
    GF(2^16) shapes (1000+200 x 64 KiB; 32768+32768 on a bounded 8 KiB-per-piece
    sample) at 1 thread and at every allowed thread (OpenMP)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib as ol
    codec, kind = ol.reference(), "reference"
    if codec is None:
        codec, kind = ol.oracle(), "port"
    try:
        gomp = ctypes.CDLL("libgomp.so.1")
    except OSError:
        gomp = None
    allowed = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    threads = max(1, min(allowed, int(os.environ.get("OMP_NUM_THREADS", allowed) or allowed)))

    def set_threads(n):
        if gomp is not None:
            gomp.omp_set_num_threads(int(n))

    cache = {}

    def shape(kk, rr, bb, loss, reps, cold):
        if (kk, bb) not in cache:
            cache[(kk, bb)] = ol.hash_bytes(7, kk, bb)
        data = cache[(kk, bb)]
        codec.encode(ol.hash_bytes(1, 300, 64), 37)  # OpenMP pool up, as after the reference's leo_init
        wce, wcd = codec.encode_work_count(kk, rr), codec.decode_work_count(kk, rr)
        lo, lr = ol.benchmark_losses(kk, rr, loss, seed=2, trial=0)
        los, lrs = set(lo), set(lr)
        res = {}
        if cold:  # fresh zero pages, one call each (the reference benchmark's methodology)
            work = np.zeros((wce, bb), dtype=np.uint8)
            a = time.perf_counter()
            codec.encode_raw(bb, kk, rr, wce, [data[i].ctypes.data for i in range(kk)],
                             [work[i].ctypes.data for i in range(wce)])
            te = time.perf_counter() - a
            dwork = np.zeros((wcd, bb), dtype=np.uint8)
            a = time.perf_counter()
            codec.decode_raw(bb, kk, rr, wcd, [None if i in los else data[i].ctypes.data for i in range(kk)],
                             [None if i in lrs else work[i].ctypes.data for i in range(rr)],
                             [dwork[i].ctypes.data for i in range(wcd)])
            td = time.perf_counter() - a
            res["cold_GBps"] = {"encode": round(kk * bb / te / 1e9, 3), "decode": round(kk * bb / td / 1e9, 3)}
        work = np.zeros((wce, bb), dtype=np.uint8)
        dwork = np.zeros((wcd, bb), dtype=np.uint8)
        pe = [work[i].ctypes.data for i in range(wce)]
        po = [data[i].ctypes.data for i in range(kk)]
        pn = [None if i in los else data[i].ctypes.data for i in range(kk)]
        pr = [None if i in lrs else work[i].ctypes.data for i in range(rr)]
        pd = [dwork[i].ctypes.data for i in range(wcd)]
        codec.encode_raw(bb, kk, rr, wce, po, pe)
        codec.decode_raw(bb, kk, rr, wcd, pn, pr, pd)
        be = bd = float("inf")
        for _ in range(reps):
            a = time.perf_counter()
            codec.encode_raw(bb, kk, rr, wce, po, pe)
            b = time.perf_counter()
            codec.decode_raw(bb, kk, rr, wcd, pn, pr, pd)
            c = time.perf_counter()
            be, bd = min(be, b - a), min(bd, c - b)
        assert all(np.array_equal(dwork[i], data[i]) for i in lo)
        res["warm_GBps"] = {"encode": round(kk * bb / be / 1e9, 3), "decode": round(kk * bb / bd / 1e9, 3)}
        return res

    # headline: warm loop for `seconds` on 1 core
    set_threads(1)
    data = ol.hash_bytes(7, k, nbytes)
    wc_e, wc_d = codec.encode_work_count(k, r), codec.decode_work_count(k, r)
    work = np.zeros((wc_e, nbytes), dtype=np.uint8)
    dwork = np.zeros((wc_d, nbytes), dtype=np.uint8)
    po = [data[i].ctypes.data for i in range(k)]
    pe = [work[i].ctypes.data for i in range(wc_e)]
    pn = [None] * k
    pr = [work[i].ctypes.data for i in range(r)]
    pd = [dwork[i].ctypes.data for i in range(wc_d)]
    assert codec.encode_raw(nbytes, k, r, wc_e, po, pe) == 0
    assert codec.decode_raw(nbytes, k, r, wc_d, pn, pr, pd) == 0
    t_enc = t_dec = 0.0
    steps = 0
    start = time.perf_counter()
    while steps < 3 or time.perf_counter() - start < seconds:
        a = time.perf_counter()
        codec.encode_raw(nbytes, k, r, wc_e, po, pe)
        b = time.perf_counter()
        codec.decode_raw(nbytes, k, r, wc_d, pn, pr, pd)
        c = time.perf_counter()
        t_enc += b - a
        t_dec += c - b
        steps += 1
    assert np.array_equal(dwork[:k], data)
    inb = k * nbytes
    detail = {"cpu_model": cpu_model(), "threads_allowed": threads,
              f"{k}+{r}x{nbytes}_1thread": shape(k, r, nbytes, k, 3, True)}
    for th in sorted({1, threads}):
        set_threads(th)
        detail[f"1000+200x65536_{th}threads"] = shape(1000, 200, 65536, 200, 3, True)
        detail[f"32768+32768x8192_{th}threads"] = shape(32768, 32768, 8192, 32768, 1, th == threads)
    set_threads(threads)
    return {"value": round(inb * steps / (t_enc + t_dec) / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": kind,
            "sample": f"{steps} encode+decode steps of {k}+{r} x {nbytes} B (full loss), warm buffers, "
                      f"{t_enc + t_dec:.1f} s on 1 core of {cpu_model()}; encode {inb * steps / t_enc / 1e9:.3f} "
                      f"GB/s, decode {inb * steps / t_dec / 1e9:.3f} GB/s",
            "detail": detail}


if __name__ == "__main__":
    main()
