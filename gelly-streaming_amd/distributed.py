"""Multi-GPU combine over torch.distributed: one process per GPU, every rank holds
a replica of the global forest and folds its own shard of each global micro-batch.

This replaces the reference's gather of per-partition summaries into a
parallelism-1 reducer (SummaryBulkAggregation.java:77-83: keyBy(partition) ->
timeWindow fold -> timeWindowAll reduce -> Merger). Union is associative and
commutative, so instead of shipping whole summaries to one task every rank ships
only the STRUCTURAL DELTA its fold made (successful hooks, plus new vertices seen
only through self-loops: O(changes), not O(V)) and folds every other rank's delta
into its replica. After finish() all replicas describe the same partition, so any
rank can answer queries / emit the Merger output.

Same protocol as the native group (include/gs_group.h), with torch collectives:
  * exchange b: fold b, stage every record (gs_delta_stage: rows + a count word
    that carries a failed signed verdict), all-gather the count words;
  * then the data of exchange b-1: all-gather exactly max-count rows per rank (the
    counts of b-1 are read on the host), and fold the other ranks' live rows
    (gs_fold_exchange_device) behind the collective on the summary's stream;
  * finish() moves and folds the last exchange.
Folding a remote delta late is exact because union commutes.
"""
import torch
import torch.distributed as dist

FAIL_BIT = 1 << 62  # count word: the sender's signed verdict failed


class DeltaExchangeFold:
    """Drives one replica through the per-batch fold + exchange.

    `summary` provides fold_device(src, dst, n=), set_delta_tracking(bool),
    delta_capacity(), delta_stage(send, cap, count, width),
    fold_exchange(recv, counts, world, rows, skip_rank, width), sync() and `stream`
    (gelly_streaming_amd.Summary does; CPU tests plug a model replica whose
    stream is None).
    """

    WIDTH = 3  # rows {a, b, w}

    def __init__(self, summary, batch, device, group=None):
        self.s = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.nccl = self.cuda and dist.get_backend(group) == "nccl"
        self.s.set_delta_tracking(True)
        self.cap = int(self.s.delta_capacity())
        self.send = [torch.empty((self.cap, self.WIDTH), dtype=torch.int64, device=self.dev) for _ in range(2)]
        self.recv = [torch.empty((self.world * self.cap, self.WIDTH), dtype=torch.int64, device=self.dev)
                     for _ in range(2)]
        self.count = torch.zeros((2, 1), dtype=torch.int64, device=self.dev)
        self.counts = torch.zeros((2, self.world), dtype=torch.int64, device=self.dev)
        if self.cuda:
            torch.cuda.synchronize(self.dev)  # the fills ran on torch's stream; stages write on the summary's
            self.stream = torch.cuda.ExternalStream(summary.stream, device=self.dev)
            self.ev_staged = [torch.cuda.Event() for _ in range(2)]
            self.ev_data = [torch.cuda.Event() for _ in range(2)]
        self.rows_received = 0
        self.live_received = 0
        self.b = 0
        self.pending = None

    # ---------------------------------------------------------------- public
    def step(self, src, dst, n):
        """Fold this rank's part of one global micro-batch, gather its record count,
        then move and fold the previous batch's records."""
        b = self.b
        self.b += 1
        k = b % 2
        self.s.fold_device(src, dst, n=n)
        self.s.delta_stage(self.send[k], self.cap, self.count[k], self.WIDTH)
        if self.nccl:
            self.ev_staged[k].record(self.stream)
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(self.ev_staged[k])
            dist.all_gather_into_tensor(self.counts[k], self.count[k], group=self.group)
        else:  # gloo: through host memory (CPU tests, several ranks on one GPU)
            self.s.sync()
            parts = [torch.empty(1, dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(parts, self.count[k].cpu(), group=self.group)
            self.counts[k].copy_(torch.cat(parts))
        if self.pending is not None:
            self._data(self.pending)
        self.pending = b

    def finish(self):
        """Move and fold the last exchange; afterwards all replicas hold the union
        of every rank's folds."""
        if self.pending is not None:
            self._data(self.pending)
            self.pending = None
        self.s.sync()
        self.b = 0

    # ---------------------------------------------------------------- internals
    def _data(self, e):
        k = e % 2
        live = [int(c) & (FAIL_BIT - 1) for c in self.counts[k].tolist()]  # (synchronises on the counts)
        rows = max(1, max(live))
        recv = self.recv[k][: self.world * rows]
        send = self.send[k][:rows]
        if self.nccl:
            cur = torch.cuda.current_stream(self.dev)
            dist.all_gather_into_tensor(recv, send, group=self.group)
            self.ev_data[k].record(cur)
            self.stream.wait_event(self.ev_data[k])  # fold behind the collective, no host sync
        else:
            self.s.sync()
            parts = [torch.empty((rows, self.WIDTH), dtype=torch.int64) for _ in range(self.world)]
            dist.all_gather(parts, send.cpu().contiguous(), group=self.group)
            recv.copy_(torch.cat(parts))
        if self.world > 1:
            self.s.fold_exchange(recv, self.counts[k], self.world, rows, self.rank, self.WIDTH)
        self.rows_received += (self.world - 1) * rows
        self.live_received += sum(live) - live[self.rank]


def tree_combine(summary, group=None):
    """Binomial-tree combine of PER-RANK PARTIAL summaries onto rank 0: the
    reference's SummaryTreeReduce / ConnectedComponentsTree
    (SummaryTreeReduce.java:68-123; `enhance` pairs partitions by f0/2 at :107 and
    reduces level by level) over torch.distributed point-to-point. At level l, rank
    r with r mod 2^(l+1) == 2^l sends its exported summary -- header
    {count, failed}, then (v, label, parity) -- to r - 2^l, which folds it as
    union(v, label) with the required parity (DisjointSet.merge, DisjointSet.java:127-131;
    Candidates.merge for the signed kind, verdict ANDed: Candidates.java:79-81).
    Same schedule as the native gs_group_tree_combine (include/gs_group.h).

    `summary` provides num_vertices(), ok(), export_labels_device(v, label, parity)
    -> count, combine_exported_device(v, label, parity, n, failed) and sync()
    (gelly_streaming_amd.Summary does; CPU tests plug a model). With gloo the
    payload is staged through host memory. Collective; returns True on the rank
    that holds the combined summary (rank 0)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    wire = dev

    def peer(r):
        return dist.get_global_rank(group, r) if group is not None else r

    xdev = getattr(summary, "device", dev)
    xdev = torch.device("cuda", xdev) if isinstance(xdev, int) else torch.device(xdev)

    step = 1
    while step < world:
        pos = rank % (2 * step)
        if pos == step:
            n = summary.num_vertices()
            cap = n + 1
            v = torch.empty(cap, dtype=torch.int64, device=xdev)
            lab = torch.empty(cap, dtype=torch.int64, device=xdev)
            par = torch.empty(cap, dtype=torch.uint8, device=xdev)
            got = summary.export_labels_device(v, lab, par)
            hdr = torch.tensor([got, 0 if summary.ok() else 1], dtype=torch.int64, device=wire)
            dist.send(hdr, peer(rank - step), group=group)
            if got:
                for t in (v[:got], lab[:got], par[:got]):
                    dist.send(t.to(wire).contiguous(), peer(rank - step), group=group)
            return False
        if pos == 0 and rank + step < world:
            src = peer(rank + step)
            hdr = torch.empty(2, dtype=torch.int64, device=wire)
            dist.recv(hdr, src, group=group)
            got, failed = int(hdr[0]), bool(hdr[1])
            bufs = [torch.empty(got, dtype=dt, device=wire) for dt in (torch.int64, torch.int64, torch.uint8)]
            for t in bufs:
                if got:
                    dist.recv(t, src, group=group)
            v, lab, par = (t.to(xdev) for t in bufs)
            if xdev.type == "cuda":
                torch.cuda.current_stream(xdev).synchronize()  # the summary's stream reads them next
            summary.combine_exported_device(v, lab, par, got, failed)
            summary.sync()
        step <<= 1
    return rank == 0
