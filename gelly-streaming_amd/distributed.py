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


def part_owner(v, world):
    """Owner rank of vertex ids (numpy int64): csrc/gs_part.hpp part_owner, bit for bit."""
    import numpy as np
    z = np.asarray(v, np.int64).view(np.uint64) ^ np.uint64(0x5851F42D4C957F2D)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return ((z >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


class PartitionedLabelCombine:
    """The owner-partitioned combine of include/gs_group.h (gs_group_create_partitioned,
    DESIGN.md section 5b) over torch.distributed: no rank replicates the graph. Each rank
    keeps a LOCAL forest of its own edges; a combine (the window end of
    SummaryBulkAggregation.java:76-83)
      1. exports (v, local root, parity) of the vertices new since the previous combine,
         bucketed by owner (part_owner), and the label pairs (a, root of a now, parity) of
         the exported roots hooked away since then;
      2. moves the rows to their owners (counts all_to_all_single, then rows
         all_to_all_single with splits);
      3. at the owner, keeps one anchor (label, parity) per vertex -- the first row's -- and
         turns every other row (v, l, p) into the pair (anchor, l, p ^ parity(anchor)); a row
         with the anchor's label and the other parity is an odd cycle;
      4. all-gathers the pairs (count words carry a failed verdict, FAIL_BIT) and folds
         every rank's pairs into every rank's LABEL forest.
    labels() = this rank's owned slice: (v, label of anchor(v), parity composed).

    `local` provides export_new() -> (v, l, p) numpy int64 arrays (marks the roots l) and
    hooked_exported() -> (a, l, p) for the marked roots hooked away since the previous call
    (and marks their roots), and failed(); `forest` provides fold(a, b, w), find(x) ->
    (root, parity) or None, and failed(). The native group runs the same steps in HIP
    kernels (csrc/gs_part_k.hip); the CPU tests plug models (tests/test_distributed_cpu.py).
    """

    WIDTH = 3

    def __init__(self, local, forest, group=None):
        self.local = local
        self.forest = forest
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.anchor = {}  # owned vertex -> (anchor label, parity of v relative to it)
        self.odd = False  # an owner saw one vertex on both sides of one label
        self.combines = 0
        self.rows_owned = 0
        self.pairs_folded = 0

    def combine(self):
        import numpy as np
        W, world = self.WIDTH, self.world
        v, l, p = self.local.export_new()
        ha, hl, hp = self.local.hooked_exported()
        own = part_owner(v, world) if len(v) else np.zeros(0, np.int64)
        order = np.argsort(own, kind="stable")
        send = torch.from_numpy(np.stack([v, l, p], 1)[order].astype(np.int64).reshape(-1, W).copy())
        scounts = torch.from_numpy(np.bincount(own, minlength=world).astype(np.int64))
        rcounts = torch.empty(world, dtype=torch.int64)
        dist.all_to_all_single(rcounts, scounts, group=self.group)
        recv = torch.empty((int(rcounts.sum()), W), dtype=torch.int64)
        dist.all_to_all_single(recv, send, output_split_sizes=rcounts.tolist(),
                               input_split_sizes=scounts.tolist(), group=self.group)
        pairs = set(zip(ha.tolist(), hl.tolist(), hp.tolist()))
        for x, lab, par in recv.tolist():
            a = self.anchor.get(x)
            if a is None:
                self.anchor[x] = (lab, par)
            elif lab != a[0]:
                pairs.add((a[0], lab, par ^ a[1]))
            elif par != a[1]:
                self.odd = True
        self.rows_owned += len(recv)
        mine = torch.tensor(sorted(pairs), dtype=torch.int64).reshape(-1, W)
        word = len(mine) | (FAIL_BIT if (self.odd or self.local.failed()) else 0)
        words = [torch.empty(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(words, torch.tensor([word], dtype=torch.int64), group=self.group)
        live = [int(w) & (FAIL_BIT - 1) for w in words]
        rows = max(1, max(live))
        pad = torch.zeros((rows, W), dtype=torch.int64)
        pad[:len(mine)] = mine
        parts = [torch.empty((rows, W), dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, pad, group=self.group)
        for r in range(world):
            if int(words[r]) & FAIL_BIT:
                self.forest.fail()
            for a, b, w in parts[r][:live[r]].tolist():
                self.forest.fold(a, b, w)
        self.pairs_folded += sum(live)
        self.combines += 1

    def ok(self):
        return not self.forest.failed()

    def labels(self):
        """This rank's owned (v, label, parity), sorted by v."""
        import numpy as np
        vs = sorted(self.anchor)
        lab, par = [], []
        for x in vs:
            a, pa = self.anchor[x]
            f = self.forest.find(a)
            root, pr = f if f is not None else (a, 0)
            lab.append(root)
            par.append(pa ^ pr)
        return np.array(vs, np.int64), np.array(lab, np.int64), np.array(par, np.int64)
