"""Multi-GPU combine: one process per GPU, every rank holds a replica of the global
forest and folds its own shard of each global micro-batch.

This replaces the reference's gather of per-partition summaries into a
parallelism-1 reducer (SummaryBulkAggregation.java:77-83: keyBy(partition) ->
timeWindow fold -> timeWindowAll reduce -> Merger). Union is associative and
commutative, so instead of shipping whole summaries to one task every rank ships
only the STRUCTURAL DELTA its fold made (successful hooks, plus new vertices that
stayed roots: O(changes), not O(V)) and folds every other rank's delta into its
replica. After each exchange all replicas describe the same partition, so any
rank can answer queries / emit the Merger output.

No host synchronisation on the per-batch path:
  * every rank sends exactly cap + 1 rows (gs_delta_stage: a header row
    {sent, queued, skip} + up to cap records) -- cap is agreed without
    communication: it starts at `first_cap` and is re-derived every `retune`
    batches from gathered headers that every rank holds identically;
  * records past cap stay queued on the device and ride with the next exchange;
  * the all-gather (RCCL, torch's current stream) waits on an event of the
    summary's stream; the fold of the other ranks' rows (gs_fold_exchange_device,
    one launch, live row counts read from the headers on the device) waits on an
    event of the collective; batch b+1 is folded before batch b's rows are
    applied, so the collective overlaps the next fold.
`finish()` applies the last batch and drains any backlog in synchronous rounds.
Folding a remote delta late is exact because union commutes.
"""
import torch
import torch.distributed as dist

SKIP = 0x80  # wire record w bit 7: padding / header row
HDR_LAG = 4  # a retune reads the gathered headers of the exchange HDR_LAG batches back
HDR_SLOTS = 8  # > HDR_LAG: header copies of successive retune periods never overwrite each other


class DeltaExchangeFold:
    """Drives one replica through the per-batch fold + exchange.

    `summary` provides fold_device(src, dst, n=), set_delta_tracking(bool),
    delta_stage(send, cap), fold_exchange(recv, world, rows, skip_rank), sync()
    and `stream` (gelly_streaming_amd.Summary does; CPU tests plug a model
    replica whose stream is None).
    """

    def __init__(self, summary, batch, device, group=None, first_cap=None, retune=4):
        self.s = summary
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.nccl = self.cuda and dist.get_backend(group) == "nccl"
        self.max_cap = 3 * int(batch)  # a fold records at most 3 per edge
        self.first_cap = min(int(first_cap) if first_cap else int(batch), self.max_cap)
        self.retune = int(retune)
        rows = self.max_cap + 1
        self.send = [torch.empty((rows, 3), dtype=torch.int64, device=self.dev) for _ in range(2)]
        self.recv = [torch.empty((self.world * rows, 3), dtype=torch.int64, device=self.dev) for _ in range(2)]
        # ring of HDR_SLOTS header copies (slot b % HDR_SLOTS = exchange hdr_batch[slot])
        self.hdr = torch.zeros((HDR_SLOTS, self.world, 3), dtype=torch.int64, pin_memory=self.cuda)
        if self.cuda:
            self.stream = torch.cuda.ExternalStream(summary.stream, device=self.dev)
            self.ev_staged = [torch.cuda.Event() for _ in range(2)]
            self.ev_done = [torch.cuda.Event() for _ in range(2)]
            self.ev_hdr = [torch.cuda.Event() for _ in range(HDR_SLOTS)]
        self.rows_received = 0
        self.cap_history = []  # cap of every exchange (diagnostics / tests)
        self._reset_state()
        self.s.set_delta_tracking(True)

    # ---------------------------------------------------------------- public
    def step(self, src, dst, n):
        """Fold this rank's part of one global micro-batch; exchange it
        asynchronously and apply the previous batch's remote rows."""
        b = self.b
        self.b += 1
        self._retune(b)  # before this exchange's own header copy can replace the lagged one
        self.s.fold_device(src, dst, n=n)
        self._exchange(b, self.cap, apply_now=False)
        self.cap_history.append(self.cap)

    def finish(self):
        """Apply the last exchange and drain every rank's backlog; afterwards all
        replicas hold the union of every rank's folds."""
        if self.pending is not None:
            self._apply(*self.pending)
            self.pending = None
        while self.b > 0:
            remaining = self._remaining_after_last()
            if remaining == 0:
                break
            b = self.b
            self.b += 1
            self._exchange(b, min(remaining, self.max_cap), apply_now=True)
        self.s.sync()
        self._reset_state()

    # ---------------------------------------------------------------- internals
    def _reset_state(self):
        self.b = 0
        self.cap = self.first_cap
        self.pending = None
        self.hdr_batch = [-1] * HDR_SLOTS
        self.last_rows = 0

    def _exchange(self, b, cap, apply_now):
        k = b % 2
        rows = cap + 1
        send = self.send[k][:rows]
        recv = self.recv[k][: self.world * rows]
        self.s.delta_stage(send, cap)
        if self.nccl:
            self.ev_staged[k].record(self.stream)
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(self.ev_staged[k])
            dist.all_gather_into_tensor(recv, send, group=self.group)
            self.ev_done[k].record(cur)
            done = self.ev_done[k]
            if (b + HDR_LAG) % self.retune == 0:  # headers for the retune HDR_LAG batches later
                self.hdr[b % HDR_SLOTS].copy_(recv.view(self.world, rows, 3)[:, 0, :], non_blocking=True)
                self.ev_hdr[b % HDR_SLOTS].record(cur)
                self.hdr_batch[b % HDR_SLOTS] = b
        else:  # gloo: stage through host memory (CPU tests, several ranks on one GPU)
            self.s.sync()
            local = send.cpu()
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local, group=self.group)
            recv.copy_(torch.cat(parts))
            if (b + HDR_LAG) % self.retune == 0:
                self.hdr[b % HDR_SLOTS].copy_(torch.stack([p[0] for p in parts]))
                self.hdr_batch[b % HDR_SLOTS] = b
            done = None
        item = (recv, done, rows)
        if apply_now:
            self._apply(*item)
        else:
            if self.pending is not None:
                self._apply(*self.pending)
            self.pending = item

    def _retune(self, b):
        # every `retune` batches all ranks re-derive cap from the same gathered headers
        # (those of exchange b - HDR_LAG, copied when that exchange ran)
        slot = (b - HDR_LAG) % HDR_SLOTS
        if b % self.retune == 0 and b >= HDR_LAG and self.hdr_batch[slot] == b - HDR_LAG:
            if self.cuda:
                self.ev_hdr[slot].synchronize()
            queued = int(self.hdr[slot, :, 1].max())
            self.cap = int(min(self.max_cap, max(4096, queued + queued // 4 + 1024)))

    def _remaining_after_last(self):
        """Largest backlog any rank still holds after the last exchange (from its
        gathered headers; synchronous -- only used by finish())."""
        if self.last_rows == 0:
            return 0
        recv = self.recv[(self.b - 1) % 2][: self.world * self.last_rows]
        if self.cuda:
            torch.cuda.synchronize(self.dev)
        h = recv.view(self.world, self.last_rows, 3)[:, 0, :].cpu()
        return int((h[:, 1] - h[:, 0]).max())

    def _apply(self, recv, done, rows):
        self.last_rows = rows
        if self.world == 1:
            return
        if done is not None:
            self.stream.wait_event(done)  # fold behind the collective, no host sync
        self.s.fold_exchange(recv, self.world, rows, self.rank)
        self.rows_received += (self.world - 1) * rows
        self.last_rows = rows


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
