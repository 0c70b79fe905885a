#!/usr/bin/env python3
"""bench.py -- streaming connected components on RMAT-26 (BASELINE.json metric).

One step = one full pass of the hot path over the whole synthetic stream:
reset the summary, fold every 2^20-edge micro-batch (SummaryBulkAggregation window
-> UpdateCC.foldEdges -> DisjointSet.union), combine across ranks after every
global micro-batch (N > 1), then the final canonical label pass (every vertex ->
min id of its component, written to HBM). Edges are generated into HBM before the
timed region (each rank its own contiguous 1/N shard of the 2^30-edge stream).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 26] [--log-batch 20]
N > 1 runs one process per GPU (RCCL). Under torch.distributed.run the ranks come
from the environment; without WORLD_SIZE, `--gpus N` starts the N ranks itself as a
child torch.distributed.run (before anything touches the GPU) and relays rank 0's
line. Every rank refuses to run unless the world that formed is exactly N.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

# Every HIP stream of a process maps onto one of GPU_MAX_HW_QUEUES hardware queues (HIP's
# default, and the GPU box's setting, is 4); streams sharing a queue run in submission
# order. The library is built for 4 (at 4 queues the one-rank
# exchange step is 44.7 ms, at 8 47.1; the plain pass 40.3 / 40.1), so the bench leaves
# the setting alone.

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_EDGE_SPARSE = 48   # 16 B edge + 2 x 12 B relabel probe + 2 x 4 B parent read


def _lib_sha16():
    import hashlib
    path = os.path.join(ROOT, "gelly-streaming_amd", "lib", "libgs_summary.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


# Calibrated ceiling of random 16-B reads from a table far larger than L2: one L2->fabric
# request each, 52-55 G requests/s on cached, uncached and fine-grained memory alike
# (tools/calib_uncached.hip, tools/calib_tlb.hip: profiles/r02_calib_uncached.txt,
# profiles/r02f_calib_tlb.txt). The fold is bound by this request rate, not by bytes.
REQUEST_CEILING_PER_S = 53.5e9


def _matching_pmc(fname, want):
    """The committed rocprofv3 PMC summary of a workload's dominant kernel
    (profiles/<fname>, written by tools/rocprof_summary.py), used only when it was taken
    of THIS library build and configuration; otherwise (None, note)."""
    path = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(path):
        return None, {"traffic_note": "no PMC profile (profiles/%s)" % fname}
    with open(path) as f:
        pm = json.load(f)
    want = dict(want, lib_sha16=_lib_sha16())
    if any(pm.get(k) != v for k, v in want.items()):
        return None, {"traffic_note": "no PMC profile of this build / configuration (profiles/%s is of %s)"
                                      % (fname, pm.get("round"))}
    return pm, {}


def _traffic_fields(pm, launches, step_s):
    """roofline.traffic = L2->fabric request bytes per launch of the dominant kernel
    (TCC_EA0_RDREQ x 128 B + WRITE_SIZE; Infinity-Cache hits included, so an upper bound
    of HBM bytes, not HBM bytes) and the request rate against the calibrated ceiling."""
    out = {"traffic_kind": "L2->fabric request bytes per launch (Infinity-Cache hits included; not HBM bytes)",
           "traffic_source": pm.get("source"), "l2_hit_rate": pm.get("l2_hit_rate"),
           "read_requests_per_launch": pm.get("read_requests_per_launch")}
    if pm.get("read_requests_per_edge") is not None:
        out["read_requests_per_edge"] = pm["read_requests_per_edge"]
    if launches and step_s:
        rps = pm["read_requests_per_launch"] * launches / step_s
        out["fabric_request_gbs_step"] = round(pm["fabric_bytes_per_launch"] * launches / step_s / 1e9, 1)
        out["read_requests_per_s_step"] = round(rps / 1e9, 2) * 1e9
        out["request_ceiling_per_s"] = REQUEST_CEILING_PER_S
        out["request_frac_step"] = round(rps / REQUEST_CEILING_PER_S, 3)
    if "sq" in pm:
        out["sq"] = {k: round(v, 4) for k, v in pm["sq"].items()}
    return int(pm["fabric_bytes_per_launch"]), out


# gs_digest of the single-GPU summary after the whole stream, per (scale, edge factor,
# seed): the constant every N > 1 replica must reproduce (computed by a one-GPU
# bench.py run of this build; the N = 1 line recomputes and checks it).
KNOWN_DIGESTS = {
    "rmat26-ef16-seed0x5eed0026": 0x961EBDC5F302C813,  # config 3 (r04a: N = 1 and the 1-rank exchange path)
    "bip-config4-clean": 0x5648FC1682105E51,           # config 4, clean stream, first-appearance ids (r04a)
    "rmat20-ef16-seed0x5eed0020": 0xDF58644480272C13,  # config 2 (r04b)
}


def _as_i64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def slice_digest_checks(part_digest, world, expected, device):
    """Self-check of the partitioned line: the digests (gs_digest's terms) of the ranks' owned
    slices, summed mod 2^64 over ranks, must equal the single-GPU summary's committed digest:
    the slices together are exactly its (v, label) set."""
    t = torch.tensor([_as_i64(part_digest)], dtype=torch.int64, device=device)
    if world > 1:
        dist.all_reduce(t)  # int64 sums wrap mod 2^64
    d = int(t.item()) & ((1 << 64) - 1)
    return {"digest": "%016x" % d, "owned_slices_digest_equals_single_gpu": None if expected is None else d == expected}


def replica_digest_checks(digest, world, expected, device):
    """Self-check of an N-rank line, outside the timed region: every
    replica's gs_digest (order-independent digest of its full (v, label) set) must be the
    same -- all-reduce MIN and MAX -- and equal to the single-GPU summary's committed
    digest for this stream. Returns the check fields."""
    lo = torch.tensor([_as_i64(digest)], dtype=torch.int64, device=device)
    hi = lo.clone()
    if world > 1:
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    out = {"replica_label_digests_equal": int(lo.item()) == int(hi.item()), "digest": "%016x" % digest}
    out["digest_equals_single_gpu"] = None if expected is None else (
        out["replica_label_digests_equal"] and digest == expected)
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", choices=["rmat-cc", "bip", "er-latency", "ingest", "dropin"], default="rmat-cc",
                   help="rmat-cc: BASELINE config 3 (the headline line); bip: config 4 (bipartiteness, "
                        "2x2^19 vertices, 2^24 edges); er-latency: config 5 (ER G(2^22, 2^26), 2^16-edge windows, "
                        "per-window latency); dropin: config 2 through the unchanged operators (C++ host mirror, "
                        "host edges, p = 1 and 8 partitions); ingest: text edge parsing")
    p.add_argument("--scale", type=int, default=26)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--log-batch", type=int, default=20)
    p.add_argument("--seed", type=lambda x: int(x, 0), default=None,
                   help="RMAT seed (default: SURVEY.md 8(d)'s, 0x5EED0020 for --scale 20 = config 2, else 0x5EED0026)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--bip-prefix-log2", type=int, default=15,
                   help="bip: edges of the prefix the quirk-exact Candidates oracle folds (O(E x components))")
    p.add_argument("--cpu-sample-log2", type=int, default=24)
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="threads of SURVEY 8(d)'s CPU leg (b): P threads fold a partition each, then CombineCC of "
                        "the partials + Merger (0: this process's CPU share, OMP_NUM_THREADS or the affinity set, "
                        "at most 16; 1: skip leg b)")
    p.add_argument("--cpu-threads-sample-log2", type=int, default=22,
                   help="edges of the threaded CPU leg's sample (the same stream's first 2^k)")
    p.add_argument("--no-profile-pass", action="store_true")
    p.add_argument("--pipeline", type=int, default=3,
                   help="pipelined windows at N=1 (gs_set_pipelining depth; 1 = strictly in order)")
    p.add_argument("--exchange", action="store_true",
                   help="run the multi-GPU delta-exchange path even at one rank (overhead measurement)")
    p.add_argument("--exchange-log-batch", type=int, default=22,
                   help="combine cadence: edges per rank (log2) between delta exchanges at N > 1 (or --exchange). "
                        "Every rank folds 2^20-edge micro-batches (SURVEY.md 8(d) config 3); the exchange runs every "
                        "4 of them by default because each exchange has a fixed host cost (DESIGN.md section 5)")
    p.add_argument("--ramp-log2", type=int, default=22,
                   help="the first 2^k edges per rank are exchanged every 2^ramp-log-batch edges (gs_group_set_ramp; "
                        "0: no ramp): fewer duplicate hook records (DESIGN.md section 5)")
    p.add_argument("--ramp-log-batch", type=int, default=20)
    p.add_argument("--capacity-log2", type=int, default=0,
                   help="relabel-table capacity hint of the CC summary (log2 vertices; 0: 2^scale)")
    p.add_argument("--rccl-max-channels", type=int, default=0,
                   help="NCCL_MAX_NCHANNELS of the RCCL communicators (0: RCCL's default). Set in this process's "
                        "environment before anything initialises HIP or RCCL, inherited by every rank; reported in "
                        "config.rccl. RCCL's collective kernels run beside the fold lanes and hold CU slots the "
                        "folds need (DESIGN.md section 5)")
    p.add_argument("--combine", choices=["auto", "replica", "partitioned"], default="auto",
                   help="N > 1 (or --exchange): replicated forests kept equal by delta all-gathers (DESIGN.md section 5), "
                        "or local forests with the owner-partitioned label combine (section 5b). auto: partitioned at "
                        "N > 1 (its per-rank replay projects above the replica's, section 5b), replica for the one-rank "
                        "--exchange line (the replica protocol's overhead measurement)")
    p.add_argument("--part-window-log2", type=int, default=0,
                   help="partitioned combine: own edges per rank between combines (log2; 0 = one combine per pass)")
    p.add_argument("--exchange-impl", choices=["native", "torch"], default="native",
                   help="native: RCCL inside libgs_summary (gs_group_*); torch: torch.distributed all-gather")
    p.add_argument("--er-mode", choices=["launch", "server"], default="server",
                   help="er-latency: which window mode `value` reports (both are measured)")
    p.add_argument("--profile-serial", action="store_true",
                   help="with --profile-only: after the timed steps, run the roofline's serialised pass (HIP events "
                        "around every k_fold launch) and stop; with --steps 0 a kernel trace then holds only that "
                        "pass, whose k_fold average is the line's fold_avg_us")
    p.add_argument("--profile-only", action="store_true",
                   help="profiling runs (tools/pmc_workload.sh): only the timed work -- no checks, no host legs, "
                        "so that every dispatch of the profiled kernel is of the measured shape")
    p.add_argument("--launch-check", action="store_true",
                   help="launcher test (CPU, gloo): form the world exactly as the bench does, print one JSON line "
                        "with the world that formed, touch no GPU")
    p.add_argument("--launch-check-digest", type=lambda x: int(x, 0), default=None,
                   help="launcher test: run the N-rank digest self-check on this synthetic digest (rank r "
                        "reports digest + r * --launch-check-digest-skew)")
    p.add_argument("--launch-check-digest-skew", type=int, default=0)
    return p.parse_args()


MULTI_RANK_WORKLOADS = ("rmat-cc", "bip")


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args):
    """`--gpus N > 1` without a launcher: start N ranks as a CHILD torch.distributed.run
    (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE from it) and return its exit code;
    rank 0's JSON line reaches this process's stdout unchanged. None when this process
    is a rank itself (WORLD_SIZE set) or N = 1. Runs before anything initialises HIP:
    the parent never touches the GPU (device_count() does not initialise it)."""
    if os.environ.get("WORLD_SIZE") or args.gpus <= 1:
        return None
    if args.workload not in MULTI_RANK_WORKLOADS:
        raise SystemExit("--workload %s is single-GPU; --gpus %d refused" % (args.workload, args.gpus))
    if not args.launch_check:
        have = torch.cuda.device_count()
        if have < args.gpus:
            raise SystemExit("--gpus %d but only %d GPU(s) visible: refusing to measure fewer" % (args.gpus, have))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    return subprocess.run(cmd, env=env).returncode


def check_world(args):
    """(world, rank, local_rank) from the launcher; exits non-zero unless the world that
    formed is exactly --gpus (a 1-rank world never stands in for N GPUs)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but the world that formed has %d rank(s)" % (args.gpus, world))
    return world, rank, local


def launch_check(args):
    """CPU rehearsal of the multi-rank launch (tests/test_bench_launch.py): gloo process
    group, world counted by an all-reduce, one JSON line on rank 0."""
    world, rank, _ = check_world(args)
    checks = None
    rccl = rccl_setting()
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        formed = int(t.item())
        # every rank would create its communicators with the same channel cap
        ch = rccl["NCCL_MAX_NCHANNELS"] or 0
        lo, hi = torch.tensor([ch]), torch.tensor([ch])
        dist.all_reduce(lo, op=dist.ReduceOp.MIN)
        dist.all_reduce(hi, op=dist.ReduceOp.MAX)
        rccl["same_on_all_ranks"] = int(lo.item()) == int(hi.item())
        if args.launch_check_digest is not None:
            d = (args.launch_check_digest + rank * args.launch_check_digest_skew) % (1 << 64)
            checks = replica_digest_checks(d, world, args.launch_check_digest, torch.device("cpu"))
        dist.destroy_process_group()
    else:
        formed = 1
    if formed != args.gpus:
        raise SystemExit("--gpus %d but %d rank(s) joined" % (args.gpus, formed))
    if rank == 0:
        line = {"launch_check": True, "n_gpus": formed, "workload": args.workload, "rccl": rccl}
        if checks is not None:
            line["self_check"] = checks
        print(json.dumps(line), flush=True)


class PartExchange:
    """bench adapter of the owner-partitioned group (gs_group_create_partitioned, DESIGN.md
    section 5b): each rank folds its shard into its LOCAL forest (pipelined micro-batches),
    combines at every window end (window 0: once, at the end of the pass) and emits its owned
    slice of the label pass."""

    def __init__(self, group, summary, window):
        self.g = group
        self.s = summary
        self.window = window

    def run(self, src, dst, n, batch):
        self.g.reset()
        step = self.window or n
        for w0 in range(0, n, step):
            for o in range(w0, min(n, w0 + step), batch):
                self.g.fold_device(src[o:], dst[o:], min(batch, n - o, w0 + step - o))
            self.g.combine()

    def labels(self, out_v, out_l):
        return self.g.labels_device(out_v, out_l)


class NativeExchange:
    """bench adapter: the same step/finish interface as DeltaExchangeFold."""

    def __init__(self, group):
        self.g = group

    def step(self, src, dst, n):
        self.g.fold_device(src, dst, n)

    def run(self, src, dst, n, batch):
        """every micro-batch of this rank's shard, looped natively"""
        self.g.fold_batches(src, dst, n, batch)

    def finish(self):
        self.g.finish()


def bench_bip(args):
    """BASELINE config 4: random bipartite stream, sides of 2^19 vertices, E = 2^24, 2^20-edge
    windows, signed (parity) union-find. Throughput on the clean stream (nothing skipped: a failed
    verdict would short-circuit the fold); verdict check on the odd-cycle variant (edges injected at
    E/8, E/4, E/2, 3E/4): at one GPU the verdict must flip in the window of the first conflicting
    edge; at N GPUs (config 4 at G = 8: one process per GPU, each rank its contiguous 1/N shard,
    signed 24-B delta rows exchanged per global micro-batch through the native group) every
    replica's final verdict must equal the truth (the remote half of a window lands one exchange
    late, so a per-window flip is only defined at one GPU)."""
    import gsamd as gs
    world, rank, local = check_world(args)
    if local >= torch.cuda.device_count():
        raise SystemExit("rank %d: LOCAL_RANK %d but %d GPU(s) visible" % (rank, local, torch.cuda.device_count()))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    grouped = world > 1 or args.exchange
    if grouped:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29534")
            dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        else:
            dist.init_process_group("nccl", device_id=dev)
    logside, E, B, seed = 19, 1 << 24, 1 << 20, 0x5EED0B1B
    per = E // world
    start = rank * per
    summ = gs.Summary("signed", device=local, capacity_hint=1 << 20)
    group = None
    if not grouped and args.pipeline > 1:
        # lanes first: every HIP stream maps onto one of GPU_MAX_HW_QUEUES (4) queues, and
        # lanes created after torch's null stream share one (effective depth 2: the r04a
        # trace of this step, profiles/r04_bip_dispatches.txt)
        summ.set_pipelining(args.pipeline)

    def stream(inject):
        """The whole config-4 stream with ids renamed in first-appearance order (SURVEY.md
        8(d): the reference's exact regime), every rank the same, before the timed region."""
        fs = torch.empty(E, dtype=torch.int64, device=dev)
        fd = torch.empty(E, dtype=torch.int64, device=dev)
        gs.gen_bip(fs, fd, 0, E, logside, seed, inject)
        torch.cuda.synchronize(dev)
        gs.relabel_first_appearance(fs, fd, 2 << logside)
        torch.cuda.synchronize(dev)
        return fs, fd

    fs, fd = stream([])
    src, dst = fs[start:start + per].clone(), fd[start:start + per].clone()
    del fs, fd
    torch.cuda.synchronize(dev)
    if grouped:
        uid = [gs.group_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        group = gs.Group(summ, uid[0], world, rank, B)
    ok = [True]

    def one_step():
        summ.reset()
        if group is not None:
            group.fold_batches(src, dst, per, B)
            group.finish()
        else:
            for o in range(0, per, B):
                summ.fold_device(src[o:], dst[o:], n=min(B, per - o))
        ok[0] = summ.ok()  # the verdict read joins every pending fold

    def barrier():
        summ.sync()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        one_step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # roofline of the signed k_fold (one GPU): HIP events around every launch over one extra
    # serialised step, the same 48 B/edge algorithmic bytes as the CC fold (the parity rides
    # in the link word); traffic from the workload's PMC profile of this build
    roof = None
    if group is None and not args.no_profile_pass:
        summ.set_profiling(True)
        one_step()
        summ.sync()
        nf, fold_ms = summ.kernel_stats("fold")
        summ.set_profiling(False)
        fold_avg_ms = fold_ms / max(nf, 1)
        per_launch = per / max(nf, 1)
        achieved = BYTES_PER_EDGE_SPARSE * per_launch / (fold_avg_ms * 1e-3) / 1e9
        step_gbs = BYTES_PER_EDGE_SPARSE * per / (el / args.steps) / 1e9
        pm, extra = _matching_pmc("pmc_bip_traffic.json", {"workload": "bip-config4", "batch": B,
                                                             "pipeline": args.pipeline})
        traffic = None
        if pm is not None:
            traffic, extra = _traffic_fields(pm, nf, el / args.steps)
        roof = {"kernel": "k_fold (signed)", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "achieved_step": round(step_gbs, 1), "frac_step": round(step_gbs / HBM_PEAK_GBS, 4),
                "bytes_per_edge": BYTES_PER_EDGE_SPARSE, "edges_per_launch": int(per_launch),
                "fold_avg_us": round(fold_avg_ms * 1e3, 2), "fold_launches": int(nf)}
        roof.update(extra)
        col = summ.colouring()
        roof["atomic_floor"] = atomic_floor(summ.num_vertices(), len(np.unique(col[1])) if col[0] else 0,
                                            el * 1e3 / args.steps)
    if args.profile_only:  # profiling run: the timed steps only
        if group is not None:
            group.close()
        summ.close()
        if world > 1 or args.exchange:
            dist.destroy_process_group()
        return
    # the clean stream's colouring, every replica against the single-GPU summary's digest
    dig = replica_digest_checks(summ.digest(), world, KNOWN_DIGESTS.get("bip-config4-clean"), dev)
    # odd-cycle variant (outside the timed region)
    inject = [E // 8, E // 4, E // 2, 3 * E // 4]
    fs, fd = stream(inject)
    src.copy_(fs[start:start + per])
    dst.copy_(fd[start:start + per])
    torch.cuda.synchronize(dev)
    if rank != 0:
        del fs, fd
    summ.reset()
    flip = None
    if group is not None:
        group.fold_batches(src, dst, per, B)
        group.finish()
        final_ok = summ.ok()
    else:
        for o in range(0, per, B):
            summ.fold_device(src[o:], dst[o:], n=B)
            if flip is None and not summ.ok():
                flip = o // B
        final_ok = summ.ok()
    oks = [bool(ok[0]), bool(final_ok)]
    if world > 1:
        v = torch.tensor(oks, dtype=torch.int32, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)  # every replica must agree below
        v2 = torch.tensor(oks, dtype=torch.int32, device=dev)
        dist.all_reduce(v2, op=dist.ReduceOp.MAX)
        agree = bool((v == v2).all().item())
        oks = [bool(x) for x in v.tolist()]
    else:
        agree = True
    line = None
    if rank == 0:
        import oracle  # checker and CPU baseline legs only
        first = oracle.bip_first_failure(fs.cpu().numpy(), fd.cpu().numpy())
        # SURVEY.md 8(a) contract (ii): does the reference's Candidates diverge from the
        # truth on this stream? Its merge is O(E x components): a capped prefix, one window.
        # With first-appearance ids it must not, and the GPU's colouring of the same prefix
        # must equal the reference's (quirk-exact restatement) string exactly.
        cap = 1 << args.bip_prefix_log2
        ps, pd = fs[:cap].cpu().numpy(), fd[:cap].cpu().numpy()
        div = oracle.bip_quirk_divergence(ps, pd)
        with gs.Summary("signed", device=local, capacity_hint=cap) as pre:
            pre.fold_device(fs[:cap], fd[:cap], n=cap)
            gpu_str = oracle.canonical_candidates_string(*pre.colouring())
        c0 = time.perf_counter()
        oracle.cpu_baseline_bip(ps, pd)
        cpu_secs = time.perf_counter() - c0
        del fs, fd
        expect = None if first < 0 else first // B
        cfg = {"workload": "bip-config4", "side_vertices": 1 << logside, "edges": E, "micro_batch": B,
               "clean_stream_bipartite": oks[0], "odd_cycle_final_verdict": oks[1],
               "odd_cycle_final_verdict_truth": first < 0, "replicas_agree": agree}
        if group is None:
            cfg.update({"odd_cycle_flip_window": flip, "odd_cycle_flip_window_truth": expect,
                        "verdict_parity": flip == expect and oks[1] == (first < 0)})
        else:
            cfg.update({"verdict_parity": agree and oks[0] and oks[1] == (first < 0),
                        "parallelism": "edge-shard x%d, per-batch signed delta all-gather (native group)" % world})
        cfg["clean_stream_digest"] = dig
        cfg["rccl"] = rccl_setting() if group is not None else None
        cfg["ids"] = "first-appearance order (SURVEY.md 8(d) config 4: the reference's exact regime)"
        cfg["reference_quirk_check"] = {
            "prefix_edges": cap, "diverges": div["diverges"], "gpu_equals_reference": gpu_str == div["quirk"],
            "note": "quirk-exact Candidates restatement (oracle/gs_oracle.cpp, Candidates.java:77-192) on the first "
                    "%d edges of the odd-cycle stream in one window: diverges = its output differs from the truth; "
                    "gpu_equals_reference = the GPU summary's (ok,{comp={v=(v,sign),...}}) string of the same prefix "
                    "equals the reference's string exactly" % cap}
        cfg["verdict_parity"] = cfg["verdict_parity"] and gpu_str == div["quirk"] and not div["diverges"]
        line = {"metric": "edges/sec for streaming bipartiteness (config 4)", "value": round(E * args.steps / el, 1),
                "unit": "edges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(el * 1e3 / args.steps, 3), "higher_is_better": True, "scaling": "strong",
                "vs_baseline": None, "dtype": "int64", "data": "synthetic", "config": cfg,
                "cpu_baseline": {"value": round(cap / cpu_secs, 1), "unit": "edges/s", "cores": 1, "kind": "port",
                                 "sample": "first %d edges of the odd-cycle stream, Candidates.merge per edge "
                                           "(quirk-exact restatement, O(E x components)), 1 thread, %.2f s"
                                           % (cap, cpu_secs)}}
        if roof is not None:
            line["roofline"] = roof
        print(json.dumps(line), flush=True)
    if group is not None:
        group.close()
    summ.close()
    if world > 1 or args.exchange:
        dist.destroy_process_group()


def bench_er_latency(args):
    """BASELINE config 5: Erdos-Renyi G(n = 2^22, m = 2^26), 1024 windows of 2^16 edges. Per
    window: fold (delta tracking on) + delta export into device memory (the records the
    Merger/combine consumes) + completion; host steady-clock latency per window, p50/p99.
    Two ways to run a window, both timed on this box: one fused launch per window
    (gs_fold_take_device), and the resident window server (gs_set_window_server: one
    persistent launch, windows posted through host-mapped memory). `value` is the p50 of
    --er-mode (default server). The line checks itself: both modes' summaries must be
    equal (device lookups of every vertex) and the first 8 windows oracle-exact."""
    import gsamd as gs
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    logn, E, B, seed = 22, 1 << 26, 1 << 16, 0x5EED00E5
    summ = gs.Summary("cc", device=0, capacity_hint=1 << (args.capacity_log2 or logn))
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_er(src, dst, 0, E, logn, seed, True, stream=summ.stream)
    summ.set_delta_tracking(True)
    cap = 3 * B + 16
    rec = torch.empty(cap * 3, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    summ.sync()
    # the C ABI called as the JNI glue calls it: raw addresses, arguments prepared once
    import ctypes
    ps, pd, prec, pcnt = src.data_ptr(), dst.data_ptr(), rec.data_ptr(), cnt.data_ptr()
    take = gs.lib().gs_fold_take_device
    k_host = ctypes.c_uint64()
    k_ref = ctypes.byref(k_host)
    res = {}
    lat_of = {}
    for mode in ("launch", "server"):
        summ.set_window_server(mode == "server")
        for step in range(args.warmup + 1):
            summ.reset()
            lat = []
            wrec = []
            nrec = 0
            for o in range(0, E, B):
                t0 = time.perf_counter()
                # one window: fold (tracked) + delta records into device memory + completion
                rc = take(summ._h, ps + 8 * o, pd + 8 * o, B, prec, cap, pcnt, k_ref)
                lat.append(time.perf_counter() - t0)
                if rc:
                    raise gs.GSError(rc, gs.lib().gs_last_error().decode())
                nrec += k_host.value
                wrec.append(k_host.value & ((1 << 62) - 1))
        lat = np.array(lat) * 1e6
        lat_of[mode] = lat
        rec_of = np.array(wrec, np.float64)  # records per window (hooks + self-loop vertices ~ inserts)
        res[mode] = {"p50_us": round(float(np.percentile(lat, 50)), 2), "p99_us": round(float(np.percentile(lat, 99)), 2),
                     "max_us": round(float(lat.max()), 2), "total_ms": round(lat.sum() * 1e-3, 3),
                     "edges_per_s": round(E / (lat.sum() * 1e-6), 1), "delta_records": nrec}
        if mode == "server":
            res[mode]["server"] = summ.window_server_stats()
        # keep this mode's final summary for the cross-check
        nv = summ.num_vertices()
        v = torch.empty(nv + 1, dtype=torch.int64, device=dev)
        lab = torch.empty(nv + 1, dtype=torch.int64, device=dev)
        summ.export_labels_device(v, lab)
        res[mode]["_v"], res[mode]["_lab"], res[mode]["_nv"] = v[:nv], lab[:nv], nv
    # self-check: the two modes' summaries are equal (every vertex looked up on the device)
    got = torch.empty_like(res["launch"]["_v"])
    fnd = torch.empty(res["launch"]["_nv"], dtype=torch.uint8, device=dev)
    summ.find_labels_device(res["launch"]["_v"], got, fnd)
    summ.sync()
    agree = (res["launch"]["_nv"] == res["server"]["_nv"] and bool(fnd.all().item()) and
             bool(torch.equal(got, res["launch"]["_lab"])))
    for m in res.values():
        for k in ("_v", "_lab", "_nv"):
            m.pop(k)
    # Latency floors of a window, the p50 is read against them:
    #  * hand-off floor: the same mode with 64-edge windows (one workgroup's dependent chain
    #    + the post/poll hand-off), 1024 windows from the stream's start, a fresh summary;
    #  * request floor: the window's fabric requests at the calibrated ceiling (>= one per
    #    endpoint probe: 2 x 2^16 requests at 53.5 G/s).
    summ.set_window_server(args.er_mode == "server")
    summ.reset()
    tiny = []
    for w in range(E // B):
        o = w * B
        t0 = time.perf_counter()
        take(summ._h, ps + 8 * o, pd + 8 * o, 64, prec, cap, pcnt, k_ref)
        tiny.append(time.perf_counter() - t0)
    handoff_us = float(np.percentile(np.array(tiny) * 1e6, 50))
    request_us = 2.0 * B / REQUEST_CEILING_PER_S * 1e6
    sel_lat = lat_of[args.er_mode]
    p99v = float(np.percentile(sel_lat, 99))
    slow = np.nonzero(sel_lat >= p99v)[0]
    # The young windows' floor: each record of a window is a vertex it
    # inserted and hooked (or a self-loop's new vertex): >= 2 memory-side atomics each (key
    # CAS, hook CAS) at the calibrated random-CAS rate, on top of the hand-off floor.
    young_rec = float(rec_of[:64].mean())
    young_floor = handoff_us + 2.0 * young_rec / ATOMIC_CAS64_PER_S * 1e6
    young_p50 = float(np.percentile(sel_lat[:64], 50))
    tail = {"p50_us_first_64_windows": round(young_p50, 2),
            "p50_us_windows_64_on": round(float(np.percentile(sel_lat[64:], 50)), 2),
            "p99_us_windows_64_on": round(float(np.percentile(sel_lat[64:], 99)), 2),
            "p99_over_p50_windows_64_on": round(float(np.percentile(sel_lat[64:], 99)) /
                                                float(np.percentile(sel_lat[64:], 50)), 3),
            "p99_windows_index_median": int(np.median(slow)) if len(slow) else None,
            "p99_windows_in_first_64": int((slow < 64).sum()), "p99_windows": int(len(slow)),
            "records_per_window_first_64": round(young_rec, 1),
            "records_per_window_64_on": round(float(rec_of[64:].mean()), 1),
            "young_window_floor_us": round(young_floor, 2),
            "young_p50_over_floor": round(young_p50 / young_floor, 3),
            "note": "where the slowest 1%% of windows sit in the stream: the young table's windows insert most "
                    "of their endpoints (CAS + vertex-list append per new vertex); their floor = the hand-off "
                    "floor + 2 memory-side atomics per record at the calibrated %.1f G CAS/s" %
                    (ATOMIC_CAS64_PER_S / 1e9)}
    floor_us = max(handoff_us, request_us)
    roof = {"kernel": "k_window_server" if args.er_mode == "server" else "k_fold<false, true, true>",
            "bound": "latency", "achieved": None, "peak": None, "unit": "us", "frac": None, "traffic": None,
            "achieved_p50_us": res[args.er_mode]["p50_us"], "floor_us": round(floor_us, 2),
            "frac_floor_over_p50": round(floor_us / res[args.er_mode]["p50_us"], 3),
            "handoff_floor_us": round(handoff_us, 2), "request_floor_us": round(request_us, 2),
            "note": "latency path: the bound is the larger of the measured 64-edge-window latency of the same mode "
                    "(dependent chain + hand-off) and the window's request floor (2 requests per edge at the "
                    "calibrated 53.5 G/s); frac_floor_over_p50 = floor / p50"}
    import oracle  # checker and CPU baseline legs only
    nchk = 8
    summ.set_window_server(args.er_mode == "server")
    summ.reset()
    for o in range(0, nchk * B, B):
        take(summ._h, ps + 8 * o, pd + 8 * o, B, prec, cap, pcnt, k_ref)
    v8, l8 = summ.labels()
    ov, olab = oracle.cc_labels(src[:nchk * B].cpu().numpy(), dst[:nchk * B].cpu().numpy())
    prefix_ok = bool(np.array_equal(v8, ov) and np.array_equal(l8, olab))
    nw = 64  # CPU baseline leg only: the 1-thread restatement on the first 64 windows
    cl = oracle.cpu_window_latency_cc(src[:nw * B].cpu().numpy(), dst[:nw * B].cpu().numpy(), B) * 1e6
    cpu = {"value": round(float(np.percentile(cl, 50)), 2), "unit": "us", "cores": 1, "kind": "port",
           "p99_us": round(float(np.percentile(cl, 99)), 2),
           "sample": "first %d windows of the same stream, DisjointSet.union per edge + CombineCC/Merger per "
                     "window (oracle/gs_oracle.cpp), 1 thread, %.1f s" % (nw, cl.sum() * 1e-6)}
    sel = res[args.er_mode]
    line = {"metric": "per-window latency p50 (us) for streaming CC on ER (config 5)",
            "value": sel["p50_us"], "unit": "us", "n_gpus": 1, "steps": 1,
            "warmup": args.warmup, "ms_per_step": sel["total_ms"], "higher_is_better": False,
            "scaling": "strong", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": "er-latency-config5", "n": 1 << logn, "edges": E, "micro_batch": B,
                       "windows": E // B, "capacity_hint": 1 << (args.capacity_log2 or logn),
                       "mode": args.er_mode, "p50_us": sel["p50_us"], "p99_us": sel["p99_us"],
                       "max_us": sel["max_us"], "edges_per_s": sel["edges_per_s"],
                       "delta_records": sel["delta_records"], "modes": res,
                       "modes_agree": agree, "first_%d_windows_oracle_exact" % nchk: prefix_ok, "tail": tail,
                       "per_window": "fold + delta export to device + completion (host steady clock; "
                                     "gs_fold_take_device; launch = one fused launch per window, server = the "
                                     "resident window server)"},
            "roofline": roof,
            "cpu_baseline": cpu}
    print(json.dumps(line), flush=True)
    summ.close()


def bench_ingest(args):
    """Text edge ingest: 2^24 RMAT-26 edges as "src dst\\n" text
    (sparse 64-bit ids, ~640 MB). Device leg: text resident in HBM -> gs_parse_edges_device
    (one pass, k_parse_fused) -> int64 src/dst. Host leg: gs_fold_text from host memory
    (pinned staging over PCIe, parse, fold) into a CC summary."""
    import gsamd as gs
    import oracle  # input formatting + CPU baseline leg only
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    E = 1 << 24
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_rmat(src, dst, 0, E, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    text_h = oracle.format_edges(hs, hd, 0)
    text = torch.from_numpy(text_h).to(dev)
    ps = torch.empty(E, dtype=torch.int64, device=dev)
    pd = torch.empty(E, dtype=torch.int64, device=dev)
    for _ in range(args.warmup):
        gs.parse_edges_device(text, ps, pd)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n, bad = gs.parse_edges_device(text, ps, pd)
    el = (time.perf_counter() - t0) / args.steps
    if args.profile_only:  # profiling run: the device-resident parses only
        return
    ok = n == E and bad == -1 and bool(torch.equal(ps, src)) and bool(torch.equal(pd, dst))
    nbytes = int(text.numel())
    alg = nbytes + 16 * E  # text read once + int64 pair written per edge
    # the parse kernel's own duration, HIP events around it inside gs_parse_edges_device
    # (an extra pass after the timed region: the events add a synchronisation per parse)
    gs.parse_set_profiling(True)
    for _ in range(max(3, args.steps)):
        gs.parse_edges_device(text, ps, pd)
    k_us_tot, k_n = gs.parse_profile()
    gs.parse_set_profiling(False)
    k_us = k_us_tot / max(k_n, 1)
    with gs.Summary("cc", device=0, capacity_hint=1 << 24) as summ:
        th = bytes(text_h)
        t1 = time.perf_counter()
        nf = summ.fold_text(th)
        summ.sync()
        host_el = time.perf_counter() - t1
    m = 1 << 20
    sample = bytes(text_h[: int(np.searchsorted(np.cumsum(text_h == 10), m)) + 1])
    c0 = time.perf_counter()
    oracle.parse_edges(sample, 0)
    cpu_el = time.perf_counter() - c0
    roof = {"kernel": "k_parse_fused (one pass: decoupled look-back over the tiles' line counts)", "bound": "hbm",
            "achieved": round(alg / k_us / 1e3, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg / k_us / 1e3 / HBM_PEAK_GBS, 4), "traffic": None,
            "kernel_avg_us": round(k_us, 2), "kernel_launches_timed": k_n,
            "achieved_wall": round(alg / el / 1e9, 1), "frac_wall": round(alg / el / 1e9 / HBM_PEAK_GBS, 4),
            "note": "algorithmic bytes = text + 16 B/edge per parse; achieved = those bytes / the parse kernel's "
                    "average duration (HIP events around k_parse_fused, gs_parse_set_profiling, an untimed pass); "
                    "achieved_wall = the same bytes / the timed per-call wall time (launches, the result kernel "
                    "and the host's poll of the mapped result included)"}
    pm, extra = _matching_pmc("pmc_ingest_traffic.json", {"workload": "ingest-rmat26-text"})
    if pm is not None:  # the parse's fabric bytes (+ a count pass's, two-pass builds), its VALU/LDS activity
        t_parse, extra = _traffic_fields(pm, 0, 0)
        t_count = int(pm.get("count_lines", {}).get("fabric_bytes_per_launch", 0))
        roof["traffic"] = t_parse + t_count
        extra["traffic_%s" % pm.get("kernel", "k_parse")] = t_parse
        extra["%s_avg_us_rocprof" % pm.get("kernel", "k_parse")] = pm.get("avg_us_rocprof")
        if t_count:
            extra["traffic_k_count_lines"] = t_count
            extra["k_count_lines_avg_us_rocprof"] = pm.get("count_lines", {}).get("avg_us_rocprof")
    roof.update(extra)
    line = {"metric": "text edge ingest: edges/sec parsed from device-resident text", "value": round(E / el, 1),
            "unit": "edges/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el * 1e3, 3), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic",
            "config": {"workload": "ingest-rmat26-text", "edges": E, "text_bytes": nbytes, "parity": ok,
                       "text_GBps": round(nbytes / el / 1e9, 1),
                       "host_fold_text_edges_per_s": round(nf / host_el, 1),
                       "host_fold_text_GBps": round(nbytes / host_el / 1e9, 2)},
            "roofline": roof,
            "cpu_baseline": {"value": round(m / cpu_el, 1), "unit": "edges/s", "cores": 1, "kind": "port",
                             "sample": "first 2^20 lines, split + Long.parseLong restatement (oracle/gs_oracle.cpp)"}}
    print(json.dumps(line), flush=True)


def bench_dropin(args):
    """SURVEY.md 8(f) row 1 / VERDICT r1 item 3: BASELINE config 2 (RMAT-20, 2^24 edges,
    2^20-edge windows) through the reference's UNCHANGED operators on the C++ host mirror
    (gelly-streaming_amd/host/gelly_streaming.hpp): per edge UpdateCC.foldEdges ->
    DisjointSet.union (buffered), per (partition, window) a fresh initial value (pooled
    handle, gs_reset), per window CombineCC of the partials and the Merger -- the call
    sequence Flink issues through the JNI glue. Edges in host memory
    (PCIe-inclusive). p = 1 and 8 partitions; final labels checked against the oracle."""
    import subprocess
    import tempfile
    import oracle  # checker and CPU baseline legs only
    exe = os.path.join(ROOT, "gelly-streaming_amd", "host", "bin", "dropin_bench")
    scale, logE, logW, seed = 20, 24, 20, 0x5EED0020
    s, d = oracle.rmat_edges(seed, scale, 0, 1 << logE, True)
    ov, olab = oracle.cc_labels(s, d)
    runs = {}
    for p in (1, 8):
        best = None
        for _ in range(max(1, args.steps)):
            with tempfile.NamedTemporaryFile(suffix=".bin") as f:
                r = subprocess.run([exe, str(scale), hex(seed), str(logE), str(logW), str(p), f.name],
                                   capture_output=True, text=True, timeout=300)
                if r.returncode != 0:
                    raise SystemExit("dropin_bench failed: " + r.stderr[-2000:])
                res = json.loads(r.stdout.strip().splitlines()[-1])
                lab = np.fromfile(f.name, dtype=np.int64).reshape(-1, 2)
            res["parity"] = bool(np.array_equal(lab[:, 0], ov) and np.array_equal(lab[:, 1], olab))
            if best is None or res["seconds"] < best["seconds"]:
                best = res
        runs[p] = best
    cpu = None
    if not args.no_cpu_baseline:
        secs1 = oracle.cpu_baseline_cc(s, d, 1 << logW, threads=1)
        cpu = {"value": round((1 << logE) / secs1, 1), "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": "the same 2^%d edges, 2^%d-edge windows: DisjointSet.union per edge + CombineCC/Merger per "
                         "window (oracle/gs_oracle.cpp), 1 thread, %.1f s" % (logE, logW, secs1)}
    line = {"metric": "edges/sec through the drop-in operators (config 2, host edges)",
            "value": round(runs[1]["edges_per_s"], 1), "unit": "edges/s", "n_gpus": 1, "steps": args.steps,
            "warmup": 0, "ms_per_step": round(runs[1]["seconds"] * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int64", "data": "synthetic",
            "config": {"workload": "dropin-rmat20-config2", "edges": 1 << logE, "window": 1 << logW,
                       "p1": runs[1], "p8": runs[8], "parity": runs[1]["parity"] and runs[8]["parity"],
                       "path": "C++ host mirror: SummaryBulkAggregation.run -> ConnectedComponents (UpdateCC, "
                               "CombineCC, Merger) over GPU DisjointSet summaries from a handle pool; wall time "
                               "includes per-edge buffering and PCIe"},
            "cpu_baseline": cpu}
    print(json.dumps(line), flush=True)


ATOMIC_CAS64_PER_S = 26.07e9  # random 64-bit CAS over a 2 GiB table (profiles/r01_calib_atomic.log)


def atomic_floor(vertices, components, step_ms):
    """The memory-side atomics a pass cannot avoid: one key CAS per vertex
    inserted and one hook CAS per union that joins two trees (vertices - components), at the
    calibrated random-CAS rate. A young table's micro-batches are bound by these, not by the
    read-request rate the steady batches run at."""
    n = 2 * int(vertices) - int(components)
    floor_ms = n / ATOMIC_CAS64_PER_S * 1e3
    return {"atomics_min_per_step": n, "vertices": int(vertices), "components": int(components),
            "ceiling_per_s": ATOMIC_CAS64_PER_S, "floor_ms": round(floor_ms, 4),
            "floor_frac_of_step": round(floor_ms / step_ms, 4), "source": "profiles/r01_calib_atomic.log"}


def rccl_setting():
    """config.rccl: the channel cap every communicator of this process was created with (the env
    RCCL reads at communicator creation; None = RCCL's default)."""
    v = os.environ.get("NCCL_MAX_NCHANNELS")
    return {"NCCL_MAX_NCHANNELS": int(v) if v else None}


def native_stdout_to_stderr():
    """RCCL prints a version banner ("RCCL version : ...", "Librccl path : ...") on the process's
    stdout when a communicator is created, ahead of the one JSON line the contract allows on
    stdout. Native code gets fd 1 pointed at stderr; this script's own prints keep the real
    stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(real, "w", buffering=1)


def main():
    args = parse()
    if args.rccl_max_channels > 0:
        # before anything touches HIP or RCCL (the ranks of self_launch inherit it, and parse it again)
        os.environ["NCCL_MAX_NCHANNELS"] = str(args.rccl_max_channels)
    if args.seed is None:
        args.seed = 0x5EED0020 if args.scale == 20 else 0x5EED0026
    rc = self_launch(args)
    if rc is not None:  # this process only launched the ranks
        sys.exit(rc)
    native_stdout_to_stderr()  # in the rank processes (self_launch's children inherit the real stdout)
    if args.launch_check:
        return launch_check(args)
    world, rank, local = check_world(args)
    if args.workload == "dropin":
        return bench_dropin(args)
    if args.workload == "ingest":
        return bench_ingest(args)
    if args.workload == "bip":
        return bench_bip(args)
    if args.workload == "er-latency":
        return bench_er_latency(args)
    if local >= torch.cuda.device_count():
        raise SystemExit("rank %d: LOCAL_RANK %d but %d GPU(s) visible" % (rank, local, torch.cuda.device_count()))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.exchange:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
        else:
            dist.init_process_group("nccl", device_id=dev)

    import gsamd as gs
    from gelly_streaming_amd.distributed import DeltaExchangeFold

    E = (1 << args.scale) * args.edge_factor
    grouped = world > 1 or args.exchange
    if args.combine == "auto":
        args.combine = "partitioned" if world > 1 else "replica"
    part = grouped and args.combine == "partitioned"
    B = 1 << (args.exchange_log_batch if grouped and not part else args.log_batch)
    per = E // world
    start = rank * per
    nbatch = (per + B - 1) // B

    xlog = args.scale - 1  # capacity hint: RMAT's distinct endpoints are about half the id space (32.8 M of 2^26)
    summ = gs.Summary("cc", device=local, capacity_hint=1 << (args.capacity_log2 or xlog))
    st = summ.stream
    src = torch.empty(per, dtype=torch.int64, device=dev)
    dst = torch.empty(per, dtype=torch.int64, device=dev)
    gs.gen_rmat(src, dst, start, per, args.scale, args.seed, True, stream=st)
    summ.sync()
    # final label pass output (device): at most min(2^scale, 2E) vertices
    vcap = min(1 << args.scale, 2 * E) + 16
    out_v = torch.empty(vcap, dtype=torch.int64, device=dev)
    out_l = torch.empty(vcap, dtype=torch.int64, device=dev)
    xch = None
    if part:
        uid = [gs.group_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        pwin = (1 << args.part_window_log2) if args.part_window_log2 else 0
        xch = PartExchange(gs.PartGroup(summ, uid[0], world, rank, 1 << (args.capacity_log2 or xlog), pwin), summ,
                           pwin)
        if args.pipeline > 1:  # (windowed: tracked folds pipeline too, the combine joins the lanes)
            summ.set_pipelining(args.pipeline)
    elif world > 1 or args.exchange:
        if args.exchange_impl == "native":
            uid = [gs.group_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            xch = NativeExchange(gs.Group(summ, uid[0], world, rank, B))
            xch.g.set_ramp(1 << args.ramp_log2 if args.ramp_log2 else 0, 1 << args.ramp_log_batch)
        else:
            xch = DeltaExchangeFold(summ, B, dev)

    if xch is None and args.pipeline > 1:
        summ.set_pipelining(args.pipeline)
    nlabels = [0]

    def one_step():
        if isinstance(xch, PartExchange):  # (reset inside: local forest, owner table, label forest)
            xch.run(src, dst, per, B)
            nlabels[0] = xch.labels(out_v, out_l)
            return
        summ.reset()
        if isinstance(xch, NativeExchange):
            xch.run(src, dst, per, B)
        else:
            for b in range(nbatch):
                o = b * B
                n = min(B, per - o)
                if xch is None:
                    summ.fold_device(src[o:], dst[o:], n=n)
                else:
                    xch.step(src[o:], dst[o:], n)
        if xch is not None:
            xch.finish()
        if world > 1:  # replicas are equal: each rank emits its 1/N slot range of the label pass
            nlabels[0] = summ.export_labels_part_device(rank, world, out_v, out_l)
        else:
            nlabels[0] = summ.export_labels_device(out_v, out_l)  # canonical label pass (syncs)

    def barrier():
        summ.sync()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        one_step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.profile_only:  # profiling / tracing run: the timed steps only
        if args.profile_serial and not grouped:  # (+ the roofline's serialised pass)
            summ.set_profiling(True)
            one_step()
            summ.sync()
            nf, fold_ms = summ.kernel_stats("fold")
            summ.set_profiling(False)
            print(json.dumps({"serial_pass_fold_launches": int(nf), "fold_avg_us": round(fold_ms * 1e3 / max(nf, 1), 2)}),
                  flush=True)
        if isinstance(xch, (NativeExchange, PartExchange)):
            xch.g.close()
        summ.close()
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    total_edges = E * args.steps
    value = total_edges / elapsed
    labelled = nlabels[0]
    checks = {}
    # every replica's (v, label) set -- not only its size -- against the single-GPU
    # summary's committed digest
    stream_key = "rmat%d-ef%d-seed%#x" % (args.scale, args.edge_factor, args.seed)
    if isinstance(xch, PartExchange):
        checks.update(slice_digest_checks(gs.digest_rows(out_v[:labelled], out_l[:labelled]), world,
                                          KNOWN_DIGESTS.get(stream_key), dev))
    else:
        checks.update(replica_digest_checks(summ.digest(), world, KNOWN_DIGESTS.get(stream_key), dev))
    checks["digest_stream"] = stream_key
    if isinstance(xch, (NativeExchange, PartExchange)):  # the world RCCL formed (ncclCommCount, both communicators)
        cc, dc = xch.g.comm_ranks()
        checks["rccl_comm_ranks"] = [cc, dc]
        checks["rccl_world_ok"] = cc == dc == world
    if world > 1:  # vertices labelled by all ranks' slices (outside the timed region)
        c = torch.tensor([labelled], dtype=torch.int64, device=dev)
        dist.all_reduce(c)
        labelled = int(c.item())
        if not part:  # every replica holds the same vertex count, and the slices cover it exactly
            nv = summ.num_vertices()
            lo = torch.tensor([nv], dtype=torch.int64, device=dev)
            hi = torch.tensor([nv], dtype=torch.int64, device=dev)
            dist.all_reduce(lo, op=dist.ReduceOp.MIN)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX)
            checks["replicas_same_vertex_count"] = int(lo.item()) == int(hi.item()) == labelled
    else:  # the label pass covers every distinct endpoint of the stream (4 slices of the id space)
        distinct = 0
        for lo_bits in range(4):
            parts = [x[(x & 3) == lo_bits] for x in (src, dst)]
            distinct += int(torch.unique(torch.cat(parts)).numel())
            del parts
        checks["vertices_equal_distinct_endpoints"] = distinct == labelled
    if rank == 0:  # the stream's first 2^24 edges (rank 0's shard starts there) vs the oracle
        import oracle  # checker leg only
        m = min(1 << 24, per)
        with gs.Summary("cc", device=local, capacity_hint=1 << 20) as chk:
            for o in range(0, m, 1 << 20):
                chk.fold_device(src[o:], dst[o:], n=min(1 << 20, m - o))
            cv, cl = chk.labels()
        ov, olab = oracle.cc_labels(src[:m].cpu().numpy(), dst[:m].cpu().numpy())
        checks["prefix_%d_edges_oracle_exact" % m] = bool(np.array_equal(cv, ov) and np.array_equal(cl, olab))

    # Roofline of the dominant kernel (k_fold). Per launch: HIP events around every
    # launch on the stream it runs on, over one extra full step (profiling serialises
    # the folds, so each event pair brackets one kernel alone). Per step: the same
    # algorithmic bytes over the timed wall clock (pipelined folds, exchange, label pass).
    roof = None
    if not args.no_profile_pass:
        summ.set_profiling(True)
        one_step()
        summ.sync()
        nf, fold_ms = summ.kernel_stats("fold")
        ns, stage_ms = summ.kernel_stats("stage")
        ne, exp_ms = summ.kernel_stats("export")
        summ.set_profiling(False)
        fold_avg_ms = fold_ms / max(nf, 1)
        edges_per_launch = per / max(nf, 1) if not grouped else 1 << 20  # own micro-batches dominate
        achieved = BYTES_PER_EDGE_SPARSE * edges_per_launch / (fold_avg_ms * 1e-3) / 1e9
        step_gbs = BYTES_PER_EDGE_SPARSE * per / (elapsed / args.steps) / 1e9
        pm, extra = _matching_pmc("pmc_r20_traffic.json" if args.scale == 20 else "pmc_fold_traffic.json",
                                  {"workload": "rmat%d-cc-stream" % args.scale, "batch": B, "pipeline": args.pipeline})
        traffic = None
        if pm is not None and not grouped:  # fabric request bytes (PMC, per launch) over the pipelined step
            traffic, extra = _traffic_fields(pm, nf, elapsed / args.steps)
        roof = {"kernel": "k_fold", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "achieved_step": round(step_gbs, 1), "frac_step": round(step_gbs / HBM_PEAK_GBS, 4),
                "bytes_per_edge": BYTES_PER_EDGE_SPARSE, "edges_per_launch": int(edges_per_launch),
                "fold_avg_us": round(fold_avg_ms * 1e3, 2), "fold_launches": int(nf),
                "stage_avg_us": round(stage_ms * 1e3 / max(ns, 1), 2), "stage_launches": int(ns),
                "export_ms": round(exp_ms, 3)}
        roof.update(extra)
        if grouped:
            roof["note"] = ("exchange path: fold launches include the other ranks' gathered rows (side stream); "
                            "achieved assumes 2^20 own edges per launch")
        else:  # the label pass's output of the profile step: its distinct labels are the components
            nl = int(nlabels[0])
            roof["atomic_floor"] = atomic_floor(nl, int(torch.unique(out_l[:nl]).numel()),
                                                elapsed * 1e3 / args.steps)

    # Per-phase device time of the exchange protocol, one extra untimed
    # step with timing events around each phase (gs_group_set_phase_timing): the N > 1
    # line explains its own scaling. Max over ranks.
    phases = None
    if isinstance(xch, PartExchange) and not args.profile_only:
        xch.g.set_phase_timing(True)
        t0p = time.perf_counter()
        one_step()
        summ.sync()
        pstep = time.perf_counter() - t0p
        ps = xch.g.phase_stats()
        stp = xch.g.stats()
        xch.g.set_phase_timing(False)
        keys = sorted(k for k in ps if k not in ("combines", "own_fold_ms"))
        vals = torch.tensor([ps[k] for k in keys] + [pstep * 1e3], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        phases = {k: round(float(v), 3) for k, v in zip(keys + ["step_ms"], vals.tolist())}
        phases.update({"combines_per_rank": int(ps["combines"]), "rows_exported_rank0": stp["rows_exported"],
                       "rows_owned_rank0": stp["rows_owned"], "pairs_folded": stp["pairs_folded"],
                       "label_forest_vertices": stp["label_forest_vertices"],
                       "note": "max over ranks, one untimed step with HIP timing events around every combine phase; "
                               "alltoall and pair_gather include the wait for the other ranks"})
    if isinstance(xch, NativeExchange) and not args.profile_only:
        xch.g.set_phase_timing(True)
        t0p = time.perf_counter()
        one_step()
        summ.sync()
        pstep = time.perf_counter() - t0p
        ps = xch.g.phase_stats()
        xch.g.set_phase_timing(False)
        keys = sorted(k for k in ps if k != "exchanges")
        vals = torch.tensor([ps[k] for k in keys] + [pstep * 1e3], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        phases = {k: round(float(v), 3) for k, v in zip(keys + ["step_ms"], vals.tolist())}
        phases["exchanges_per_rank"] = ps["exchanges"]
        st_ = xch.g.stats()
        phases["records_sent_rank0"] = st_["records_sent"]
        phases["rows_received_rank0"] = st_["rows_received"]
        phases["note"] = ("max over ranks, one untimed step with HIP timing events around every phase; own-fold "
                          "time is summed over the 3 pipelining lanes (overlapping), host_wait_counts is the host's "
                          "poll for gathered counts")

    # Secondary, PCIe-inclusive figure: the stream's first 2^27 edges
    # folded from PINNED host memory through gs_fold in 2^20-edge calls (H2D copies by
    # DMA straight from the caller's buffer, then the fold) into a fresh summary, outside
    # the timed region. Never `value`.
    pcie = None
    if rank == 0 and world == 1 and xch is None and not args.profile_only:
        m = min(1 << 27, per)
        hs = torch.empty(m, dtype=torch.int64, pin_memory=True)
        hd = torch.empty(m, dtype=torch.int64, pin_memory=True)
        hs.copy_(src[:m])
        hd.copy_(dst[:m])
        torch.cuda.synchronize()
        ns_, nd_ = hs.numpy(), hd.numpy()
        with gs.Summary("cc", device=local, capacity_hint=1 << xlog) as hsum:
            for rep in range(2):  # the first pass warms the staging buffers and the table
                hsum.reset()
                hsum.sync()
                t0 = time.perf_counter()
                for o in range(0, m, 1 << 20):
                    hsum.fold(ns_[o:o + (1 << 20)], nd_[o:o + (1 << 20)])
                hsum.sync()
                pel = time.perf_counter() - t0
        pcie = {"edges_per_s": round(m / pel, 1), "edges": m, "GBps_h2d": round(16 * m / pel / 1e9, 1),
                "source": "first 2^27 edges from pinned host memory, gs_fold in 2^20-edge calls (H2D by DMA "
                          "from the caller's buffer + fold), one GPU, outside the timed region"}
        del hs, hd, ns_, nd_

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle  # CPU baseline leg only
        m = 1 << args.cpu_sample_log2
        hs = src[:m].cpu().numpy()
        hd = dst[:m].cpu().numpy()
        secs1 = oracle.cpu_baseline_cc(hs, hd, B, threads=1)
        # SURVEY.md 8(d) leg (b): P threads, each folding a 1/P partition of every window
        # (PartitionMapper + keyed fold, S/SummaryBulkAggregation.java:77-83), then CombineCC of
        # the partials and the Merger on one thread. P = this process's CPU share (the GPU box
        # exports OMP_NUM_THREADS=16; nproc there shows the whole machine). Timed on the first
        # 2^22 edges: the combines make it slower than one thread per edge (r02: 0.66 vs 0.91 M
        # edges/s), and 2^24 edges would cost ~25 s.
        p = args.cpu_threads
        if p <= 0:
            try:
                aff = len(os.sched_getaffinity(0))
            except AttributeError:
                aff = os.cpu_count() or 1
            p = min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or aff)
        cpu = {"value": round(m / secs1, 1), "unit": "edges/s", "cores": 1, "kind": "port",
               "sample": "first 2^%d edges of the same RMAT-%d stream, %d-edge windows, C++ restatement of "
                         "DisjointSet.union + CombineCC/Merger per window (oracle/gs_oracle.cpp); 1 thread %.1f s"
                         % (args.cpu_sample_log2, args.scale, B, secs1),
               "legs": {"a_1thread": {"value": round(m / secs1, 1), "cores": 1, "edges": m,
                                      "seconds": round(secs1, 2)}}}
        if p > 1:
            mp = min(m, 1 << args.cpu_threads_sample_log2)
            secsp = oracle.cpu_baseline_cc(hs[:mp], hd[:mp], B, threads=p)
            cpu["legs"]["b_partitioned"] = {"value": round(mp / secsp, 1), "cores": p, "edges": mp,
                                            "seconds": round(secsp, 2),
                                            "what": "%d threads fold a partition of every window each, then "
                                                    "CombineCC of the partials + Merger" % p}
            cpu["value_%dthreads" % p] = round(mp / secsp, 1)
            cpu["sample"] += "; leg b: %d threads (partitioned fold + CombineCC) on the first 2^%d edges, %.1f s" % (
                p, args.cpu_threads_sample_log2, secsp)
            if mp / secsp > m / secs1:  # value = the faster leg, cores = its threads
                cpu["value"], cpu["cores"] = round(mp / secsp, 1), p

    if rank == 0:
        line = {
            "metric": "edges/sec (whole node) for streaming CC on RMAT-%d" % args.scale,
            "value": round(value, 1),
            "unit": "edges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": "rmat%d-cc-stream" % args.scale, "scale": args.scale,
                       "edges": E, "micro_batch": 1 << args.log_batch if not grouped else 1 << 20,
                       "combine_every_edges_per_gpu": ((1 << args.part_window_log2) if args.part_window_log2 else per)
                       if part else 1 << args.exchange_log_batch,
                       "combine_ramp": None if part else {
                           "first_edges_per_gpu": 1 << args.ramp_log2 if args.ramp_log2 else 0,
                           "every": 1 << args.ramp_log_batch},
                       "combine": ("owner-partitioned label combine (native RCCL group), %s" % (
                           "every 2^%d own edges" % args.part_window_log2 if args.part_window_log2 else
                           "once per pass") if part else
                                   "delta exchange (native RCCL group)" if grouped else "none at 1 GPU (same cadence)"),
                       "ids": "sparse 64-bit (scrambled)",
                       "capacity_hint": 1 << (args.capacity_log2 or xlog),
                       "vertices_labelled": int(labelled), "self_check": checks, "exchange_phases": phases,
                       "pcie_inclusive": pcie,
                       "rccl": rccl_setting() if grouped else None,
                       "parallelism": ("edge-shard x%d, local forests + owner all-to-all + label-pair all-gather"
                                       % world if part else
                                       "edge-shard x%d, per-batch delta all-gather (%s)" % (world, args.exchange_impl))
                       if xch is not None else "single GPU"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if isinstance(xch, (NativeExchange, PartExchange)):
        xch.g.close()
    summ.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
