"""Multi-GPU combine: one process per GPU, every rank holds a replica of the global
forest and folds its own shard of each global micro-batch.

This replaces the reference's gather of per-partition summaries into a
parallelism-1 reducer (SummaryBulkAggregation.java:77-83: keyBy(partition) ->
timeWindow fold -> timeWindowAll reduce -> Merger). Union is associative and
commutative, so instead of shipping whole summaries to one task every rank ships
only the STRUCTURAL DELTA its fold made (new vertices, successful hooks: at most
one record per merged component, i.e. O(changes), not O(V)) and folds every other
rank's delta into its replica. After each exchange all replicas describe the same
partition, so each rank can answer queries / emit the Merger output locally.

Collectives (RCCL over xGMI for `nccl`, gloo on CPU in tests): one all-gather of
the per-rank delta counts, one all-gather of the padded (3 x max_count) int64
payload. No other data-path communication.
"""
import torch
import torch.distributed as dist


def all_gather_varlen(a, b, w, k, group=None):
    """All-gather variable-length (a[:k], b[:k], w[:k]) from every rank.
    Returns [(a_r, b_r, w_r)] per rank (views into one gathered buffer).
    With the gloo backend device tensors are staged through host memory (tests
    run several ranks on one GPU that way); with nccl (RCCL) they stay in HBM."""
    world = dist.get_world_size(group)
    if a.is_cuda and dist.get_backend(group) == "gloo":
        parts = all_gather_varlen(a[:k].cpu(), b[:k].cpu(), w[:k].cpu(), k, group)
        return [(pa.to(a.device), pb.to(a.device), pw.to(a.device)) for pa, pb, pw in parts]
    dev = a.device
    cnt = torch.tensor([int(k)], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    cnts = [int(c.item()) for c in cnts]
    m = max(cnts)
    if m == 0:
        return [(a[:0], b[:0], w[:0]) for _ in range(world)]
    payload = torch.zeros((3, m), dtype=torch.int64, device=dev)
    if k:
        payload[0, :k] = a[:k]
        payload[1, :k] = b[:k]
        payload[2, :k] = w[:k].to(torch.int64)
    outs = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(outs, payload, group=group)
    return [(o[0, :c], o[1, :c], o[2, :c].to(torch.uint8)) for o, c in zip(outs, cnts)]


class DeltaExchangeFold:
    """Drives one replica through the per-batch fold + exchange.

    `summary` provides: fold_device(src, dst, n=, w=), set_delta_tracking(bool),
    take_delta_device(a, b, w) -> count, sync(), and optionally `stream`
    (gelly_streaming_amd.Summary does; the CPU tests plug an oracle-backed replica).
    """

    def __init__(self, summary, delta_capacity, device, group=None):
        self.s = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.a = torch.empty(delta_capacity, dtype=torch.int64, device=device)
        self.b = torch.empty(delta_capacity, dtype=torch.int64, device=device)
        self.w = torch.empty(delta_capacity, dtype=torch.uint8, device=device)
        self.exchanged = 0  # delta records received from other ranks
        self.s.set_delta_tracking(True)

    def step(self, src, dst, n, w=None):
        """Fold this rank's part of one global micro-batch, then combine."""
        self.s.fold_device(src, dst, n=n, w=w)
        k = self.s.take_delta_device(self.a, self.b, self.w)
        self.s.sync()  # packed delta complete before the collective reads it
        parts = all_gather_varlen(self.a, self.b, self.w, k, self.group)
        if self.a.is_cuda:
            torch.cuda.current_stream().synchronize()  # gathered payload complete
        self.s.set_delta_tracking(False)  # applied deltas are not re-broadcast
        for r, (pa, pb, pw) in enumerate(parts):
            if r == self.rank or pa.numel() == 0:
                continue
            self.s.fold_device(pa, pb, n=pa.numel(), w=pw)
            self.exchanged += pa.numel()
        self.s.sync()  # the gathered buffers stay alive until the fold has read them
        self.s.set_delta_tracking(True)
