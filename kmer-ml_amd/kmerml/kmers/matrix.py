"""Genomes x k-mers count matrix, one block of genomes per GPU, assembled by all-gather.

The reference builds its organisms x k-mers matrix on one CPU from per-organism files
(/root/reference/kmerml/ml/features.py:28-117, ``KmerFeatureBuilder``; rows in the sorted
file order of find_files, features.py:46).  Here every rank (one process per GPU,
``torch.distributed`` with the "nccl" backend = RCCL over xGMI) counts a contiguous
block of the genome list straight into its rows of a dense ``[G, 4^k]`` uint32 matrix in
HBM, and one ``all_gather_into_tensor`` assembles the full matrix on every rank (rows
travel as saturating u4 plus an exact escape list, 8x fewer bytes over xGMI).  Row g
is genome g of the input order; column c is the k-mer with 2-bit code c (A0 C1 G2 T3,
first base most significant, i.e. lexicographic order).  Counting follows
generate.py:39-58 exactly (records shorter than k skipped, non-ACGT windows dropped).

Nothing here falls back to the CPU; ``count_fn`` exists so the sharding and assembly
logic can be exercised with the gloo backend in CPU-only tests.
"""
import os

import numpy as np

from kmerml import _native

# Wire format the last gather_rows_* call ended up using ("u4", "u8" or "u32").
LAST_WIRE = None


def _cap_override(name, cap):
    """Test knob: KMH_ESC_CAP_U4 / KMH_ESC_CAP_U8 lower an escape capacity so that the exact
    fallbacks (u4 -> u8 -> u32) can be forced on real data.  Only ever lowers the capacity:
    a lower cap changes which wire format is used, never the assembled matrix."""
    v = os.environ.get(name)
    return min(cap, max(0, int(v))) if v else cap


def _all_reduce_max(t, group):
    import torch.distributed as dist

    if t.is_cuda and dist.get_backend(group) == "gloo":   # gloo reduces host tensors
        h = t.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


def _all_gather(out, inp, group):
    import torch
    import torch.distributed as dist

    if inp.is_cuda and dist.get_backend(group) == "gloo":   # gloo gathers host tensors
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)
    return out


def shard_bounds(n_items, world, rank):
    """Contiguous block [lo, hi) of n_items for `rank` (sizes differ by at most one)."""
    lo = (n_items * rank) // world
    hi = (n_items * (rank + 1)) // world
    return lo, hi


def block_rows(n_items, world):
    """Rows per rank in the padded all-gather buffer."""
    return -(-n_items // world) if n_items else 0


def pack_genomes(genome_files, k):
    """Parse FASTA files and lay them out for kmh_count_dense_dev.

    Returns (buffer uint8, offsets uint64[G+1]); genome starts are 16-byte aligned and
    separated by non-base padding; records shorter than k are dropped
    (generate.py:44-46 with k_values = [k]).
    """
    parts, offsets, pos = [], [0], 0
    for path in genome_files:
        f = _native.FastaFile(path)
        seq, _ = f.pack(k)
        f.close()
        pad = (-(seq.size)) % 16
        parts.append(seq)
        if pad:
            parts.append(np.full(pad, ord("\n"), np.uint8))
        pos += seq.size + pad
        offsets.append(pos)  # genome g = [offsets[g], offsets[g+1]); its padding is not a base
    buf = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return buf, np.asarray(offsets, dtype=np.uint64)


def _hip_count_block(genome_files, k, device):
    import torch

    buf, offsets = pack_genomes(genome_files, k)
    dev = torch.device("cuda", device)
    d_seq = torch.from_numpy(buf).to(dev) if buf.size else torch.zeros(16, dtype=torch.uint8, device=dev)
    out = torch.empty((len(genome_files), 1 << (2 * k)), dtype=torch.int32, device=dev)
    if len(genome_files):
        ctx = _native.context(device)
        stream = torch.cuda.current_stream(dev).cuda_stream
        ctx.count_dense_dev(d_seq.data_ptr(), offsets, k, out.data_ptr(), stream)
    return out


def slot_layout(rows, cols):
    """Packed per-rank all-gather slot of the u8 assembly.

    [rows * cols saturating u8 counts][escape count u32 + 12 B pad][cap (row, col, value) u32
    triples]; returns (cap, slot_bytes).  cap allows one escape (count >= 255) per 1024 cells.
    """
    cap = _cap_override("KMH_ESC_CAP_U8", max(4096, rows * cols // 1024))
    return cap, (rows * cols + 16 + cap * 12 + 255) // 256 * 256


def slot_layout_u4(rows, cols):
    """Packed per-rank all-gather slot of the u4 assembly (the multi-GPU default).

    [rows * cols / 2 bytes: two counts per byte, values >= 15 stored as 15][escape count u32 +
    12 B pad][cap (index, value) u32 pairs, index = row * cols + col]; returns (cap,
    slot_bytes).  cap allows one escape (count >= 15) per 256 cells: uniform 100 Mbp genomes at
    k = 12 (Poisson, mean ~6) need ~1.4 per 1000.
    """
    cap = _cap_override("KMH_ESC_CAP_U4", max(4096, rows * cols // 256))
    return cap, (rows * cols // 2 + 16 + cap * 8 + 255) // 256 * 256


def escape_count(word_bytes):
    """The u32 escape counter at the head of a slot's escape area (4 uint8 device bytes), as
    an int64 tensor: read unsigned, so a count of 2^31 or more never looks negative and skips
    the overflow check (the encoders count every escape, also those past cap)."""
    import torch

    return word_bytes.view(torch.int32).to(torch.int64) & 0xFFFFFFFF


class AssembledMatrix:
    """The assembled [G, cols] count matrix on one rank, kept as the all-gathered u4 slots
    (two counts per byte + each rank's exact escape list) instead of widened u32 rows: 8x less
    HBM per rank, and no widening pass in the step.  Exact: rows(lo, hi) widens any range of
    rows on the device (kmh_rows_decode_u4_range_dev applies exactly their escapes); dense()
    widens everything.  Rows are genomes in input order (rank r holds block shard_bounds(G, W, r)
    in slot r of `recv`), as in the reference's organisms x k-mers matrix (features.py:85-117).
    A matrix that had to fall back to a dense wire format wraps the dense tensor instead."""

    def __init__(self, G, cols, world, B, recv=None, cap=0, P=0, dense=None):
        self.G, self.cols, self.world, self.B = G, cols, world, B
        self.recv, self.cap, self.P, self._dense = recv, cap, P, dense
        self.wire = "u4" if dense is None else LAST_WIRE

    @property
    def shape(self):
        return (self.G, self.cols)

    def _slot_rows(self, q):
        lo, hi = shard_bounds(self.G, self.world, q)
        return lo, hi

    def rows(self, lo, hi, stream=None):
        """Rows [lo, hi) as a new device int32 tensor (u32 counts)."""
        import torch

        if not 0 <= lo <= hi <= self.G:
            raise IndexError(f"rows [{lo}, {hi}) outside [0, {self.G})")
        if self._dense is not None:
            idx = []
            for g in range(lo, hi):
                q = self._rank_of(g)
                idx.append(q * self.B + g - self._slot_rows(q)[0])
            return self._dense[torch.tensor(idx, dtype=torch.long, device=self._dense.device)]
        dev = self.recv.device
        out = torch.empty((hi - lo, self.cols), dtype=torch.int32, device=dev)
        ctx = _native.context(dev.index)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        nib = self.B * self.cols // 2
        g = lo
        while g < hi:
            q = self._rank_of(g)
            qlo, qhi = self._slot_rows(q)
            n = min(hi, qhi) - g
            slot = self.recv.data_ptr() + q * self.P
            ctx.rows_decode_u4_range(slot, self.B, self.cols, slot + nib + 16, self.cap, slot + nib,
                                     g - qlo, n, out[g - lo:].data_ptr(), s)
            g += n
        return out

    def row(self, g):
        return self.rows(g, g + 1)[0]

    def dense(self):
        """The whole [G, cols] matrix widened to int32 (u32 counts)."""
        return self.rows(0, self.G)

    def _rank_of(self, g):
        for q in range(self.world):
            lo, hi = shard_bounds(self.G, self.world, q)
            if lo <= g < hi:
                return q
        raise IndexError(g)


def gather_rows_u4(padded, group=None, compact=False, G=None):
    """All-gather [B, cols] u32 rows (device int32 tensor) from every rank as u4 + escapes.

    Exact for any counts: values >= 15 travel in the escape list.  If any rank has more
    escapes than the slot holds, every rank falls back to the u8 path (and from there, if
    needed, to the plain u32 all-gather).  compact=True returns an AssembledMatrix of G rows
    that keeps the gathered slots (no widening); otherwise the padded [W * B, cols] rows.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    B, cols = padded.shape
    dev = padded.device
    ctx = _native.context(dev.index)
    s = torch.cuda.current_stream(dev).cuda_stream
    cap, P = slot_layout_u4(B, cols)
    nib = B * cols // 2
    send = torch.empty(P, dtype=torch.uint8, device=dev)
    ctx.rows_encode_u4(padded.data_ptr(), B, cols, send.data_ptr(), send[nib + 16:].data_ptr(),
                       cap, send[nib:].data_ptr(), s)
    n = _all_reduce_max(escape_count(send[nib:nib + 4]), group)
    if int(n.item()) > cap:
        del send
        out = gather_rows_u8(padded, group)
        return AssembledMatrix(G, cols, world, B, dense=out) if compact else out
    global LAST_WIRE
    LAST_WIRE = "u4"
    recv = _all_gather(torch.empty(world * P, dtype=torch.uint8, device=dev), send, group)
    if compact:
        return AssembledMatrix(G if G is not None else world * B, cols, world, B, recv=recv, cap=cap, P=P)
    out = torch.empty((world * B, cols), dtype=padded.dtype, device=dev)
    base = recv.data_ptr()
    for q in range(world):
        slot = base + q * P
        ctx.rows_decode_u4(slot, B, cols, slot + nib + 16, cap, slot + nib, out[q * B:].data_ptr(), s)
    return out


def gather_rows_u8(padded, group=None):
    """All-gather [B, cols] u32 rows (device int32 tensor) from every rank as u8 + escapes.

    Exact for any counts: values >= 255 travel in the escape list.  If any rank has more
    escapes than the slot holds, every rank falls back to the plain u32 all-gather.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    B, cols = padded.shape
    dev = padded.device
    ctx = _native.context(dev.index)
    s = torch.cuda.current_stream(dev).cuda_stream
    cap, P = slot_layout(B, cols)
    u8_bytes = B * cols
    send = torch.empty(P, dtype=torch.uint8, device=dev)
    ctx.rows_encode_u8(padded.data_ptr(), B, cols, send.data_ptr(), send[u8_bytes + 16:].data_ptr(),
                       cap, send[u8_bytes:].data_ptr(), s)
    n = _all_reduce_max(escape_count(send[u8_bytes:u8_bytes + 4]), group)
    global LAST_WIRE
    if int(n.item()) > cap:
        LAST_WIRE = "u32"
        del send
        return _all_gather(torch.empty((world * B, cols), dtype=padded.dtype, device=dev), padded, group)
    LAST_WIRE = "u8"
    recv = _all_gather(torch.empty(world * P, dtype=torch.uint8, device=dev), send, group)
    out = torch.empty((world * B, cols), dtype=padded.dtype, device=dev)
    base = recv.data_ptr()
    for q in range(world):
        slot = base + q * P
        ctx.rows_decode_u8(slot, B, cols, slot + u8_bytes + 16, cap, slot + u8_bytes, 1, B,
                           out[q * B:].data_ptr(), s)
    return out


def count_matrix(genome_files, k, device=None, group=None, count_fn=None, compact=False):
    """Dense [G, 4^k] count matrix of `genome_files` (torch tensor, int32 storage of u32).

    Without an initialised torch.distributed process group this counts every genome on
    one device.  With one, rank r counts block shard_bounds(G, W, r) and the blocks are
    all-gathered (u4 rows + exact escapes on the wire for k >= 3, u8 for k = 2), so every rank
    returns the full matrix in input order.
    count_fn(files, k) -> tensor [len(files), 4^k] replaces the HIP counter (tests).
    compact=True (process group, u4 wire): return an AssembledMatrix that keeps the gathered u4
    slots and widens rows on access, instead of the dense [G, 4^k] tensor.
    """
    import torch
    import torch.distributed as dist

    if not 1 <= k <= _native.MAX_DENSE_K:
        raise NotImplementedError("the dense count matrix needs 1 <= k <= 12")
    files = list(genome_files)
    G = len(files)
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    counter = count_fn or (lambda fs, kk: _hip_count_block(fs, kk, device))
    if not (dist.is_available() and dist.is_initialized()):
        return counter(files, k)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(G, world, rank)
    local = counter(files[lo:hi], k)
    B = block_rows(G, world)
    padded = torch.zeros((B, 1 << (2 * k)), dtype=local.dtype, device=local.device)
    padded[: hi - lo] = local
    if padded.is_cuda and B and padded.shape[1] % 32 == 0 and B * padded.shape[1] < 2**32 - 1:
        if compact:
            return gather_rows_u4(padded, group, compact=True, G=G)
        gathered = gather_rows_u4(padded, group)
    elif padded.is_cuda and B and padded.shape[1] % 16 == 0:
        gathered = gather_rows_u8(padded, group)
    else:
        global LAST_WIRE
        LAST_WIRE = "u32"
        gathered = _all_gather(torch.empty((world * B, 1 << (2 * k)), dtype=local.dtype, device=local.device),
                               padded, group)
    rows = [gathered[r * B: r * B + (shard_bounds(G, world, r)[1] - shard_bounds(G, world, r)[0])]
            for r in range(world)]
    return torch.cat(rows, 0) if rows else gathered[:0]


def sparse_rows(genome_files, k, canonical=True, device=None, group=None):
    """Sparse k-mer counts of this rank's block of `genome_files` (BASELINE config 5).

    For 13 <= k <= 32 the genomes are counted on the GPU with the partitioned hash-table path
    (kmh_count_sparse_dev); any other 1 <= k <= 32 genome by genome with the GPU sort path of
    kmh_count_host (dense table for k <= 12).  The 4^k columns cannot be assembled densely (4^21 ~ 4.4e12), so
    nothing is exchanged: with a torch.distributed process group, rank r counts block
    shard_bounds(G, W, r) and keeps it.  Returns (lo, rows) where rows[i] is
    (codes uint64 ascending, counts uint32) of genome lo + i.
    """
    import torch
    import torch.distributed as dist

    if not 1 <= k <= 32:
        raise NotImplementedError("sparse rows need 1 <= k <= 32 (a 64-bit code per k-mer)")
    files = list(genome_files)
    world, rank = 1, 0
    if dist.is_available() and dist.is_initialized():
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_bounds(len(files), world, rank)
    if device is None:
        device = torch.cuda.current_device()
    if hi == lo:
        return lo, []
    buf, offsets = pack_genomes(files[lo:hi], k)
    if not 13 <= k <= 32:   # outside the batched hash-table path: one GPU count per genome
        ctx = _native.context(device)
        rows = []
        for g in range(hi - lo):
            codes, counts, _ = ctx.count(buf[int(offsets[g]):int(offsets[g + 1])], k, canonical=canonical)
            order = np.argsort(codes, kind="stable")
            rows.append((codes[order], counts[order]))
        return lo, rows
    dev = torch.device("cuda", device)
    d_seq = torch.from_numpy(buf).to(dev) if buf.size else torch.zeros(16, dtype=torch.uint8, device=dev)
    out_off = _native.sparse_out_offsets(offsets, k)
    cap = max(int(out_off[-1]), 1)
    d_codes = torch.empty(cap, dtype=torch.int64, device=dev)
    d_counts = torch.empty(cap, dtype=torch.int32, device=dev)
    d_n = torch.empty(hi - lo, dtype=torch.int64, device=dev)
    ctx = _native.context(device)
    ctx.count_sparse_dev(d_seq.data_ptr(), offsets, k, canonical, d_codes.data_ptr(), d_counts.data_ptr(),
                         d_n.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    n = d_n.cpu().numpy()
    rows = []
    for g in range(hi - lo):
        a = int(out_off[g])
        # codes use all 64 bits at k = 32: order them as unsigned (torch sorts int64 signed)
        c = d_codes[a:a + int(n[g])].cpu().numpy().view(np.uint64)
        order = np.argsort(c, kind="stable")
        rows.append((c[order], d_counts[a:a + int(n[g])].cpu().numpy().view(np.uint32)[order]))
    return lo, rows


def split_bounds(n, world, rank, k, align=16):
    """Rank `rank`'s slice of a packed genome of n bytes split across `world` ranks.

    Returns (a, b, e): the rank counts the windows that start in [a, b) from the bytes [a, e),
    e = min(n, b + k - 1) (a (k - 1)-byte halo past b).  a and b are multiples of `align` (the
    device counter wants 16-byte aligned starts), the last rank ends at n, so the ranks' [a, b)
    tile [0, n) and every window is counted by exactly one rank.
    """
    a = (n * rank // world) // align * align
    b = n if rank == world - 1 else (n * (rank + 1) // world) // align * align
    return a, b, min(n, b + k - 1)


def _hip_count_slice(sl, k, device):
    import torch

    dev = torch.device("cuda", device)
    out = torch.zeros((1, 1 << (2 * k)), dtype=torch.int32, device=dev)
    if sl.size >= k:
        d_seq = torch.from_numpy(np.ascontiguousarray(sl)).to(dev)
        ctx = _native.context(device)
        ctx.count_dense_dev(d_seq.data_ptr(), np.array([0, sl.size], dtype=np.uint64), k, out.data_ptr(),
                            torch.cuda.current_stream(dev).cuda_stream)
    return out[0]


def count_genome_split(genome_file, k, device=None, group=None, count_fn=None):
    """Dense [4^k] count row of ONE genome counted by every rank together (SURVEY.md 8(e),
    the optional split of a genome too large for one GPU's share of the work).

    The genome is packed as for count_matrix (records shorter than k dropped, records joined
    by a non-base byte, generate.py:39-56); rank r counts the windows that start in its slice
    split_bounds(n, W, r, k) -- the slice plus a (k - 1)-byte halo -- and one all-reduce(SUM)
    over the process group (RCCL over xGMI with the "nccl" backend) adds the partial rows, so
    every rank returns the genome's full row (int32 storage of u32: the sum wraps exactly like
    u32).  Without a process group the whole genome is counted on one device.
    count_fn(uint8 slice, k) -> tensor [4^k] replaces the HIP counter (CPU tests).
    """
    import torch
    import torch.distributed as dist

    if not 1 <= k <= _native.MAX_DENSE_K:
        raise NotImplementedError("the dense count row needs 1 <= k <= 12")
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    counter = count_fn or (lambda sl, kk: _hip_count_slice(sl, kk, device))
    buf, _ = pack_genomes([genome_file], k)
    if not (dist.is_available() and dist.is_initialized()):
        return counter(buf, k)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    a, _, e = split_bounds(buf.size, world, rank, k)
    row = counter(buf[a:e], k).clone()
    if dist.get_backend(group) == "gloo" and row.is_cuda:   # gloo reduces host tensors
        host = row.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        return host.to(row.device)
    dist.all_reduce(row, op=dist.ReduceOp.SUM, group=group)
    return row


# ---------------------------------------------------------------- sparse matrix, column-sharded
class ShardedSparseMatrix:
    """One rank's column shard of the organisms x k-mers count matrix for sparse k (config 5).

    The reference's matrix (features.py:85-117, ``_build_matrix``) has one column per label in
    the sorted union of every organism's labels and a 0 wherever an organism lacks one.  At
    k = 21 that union is ~10^10 columns over a 128-genome batch, so no rank holds it: rank q owns
    the codes [lo_code, hi_code) (contiguous code ranges chosen to balance the entries) and holds
    every organism's counts of those codes in CSR form:

      columns  uint64 [ncols]   the sorted union of the organisms' codes in the range
      indptr   int64  [G + 1]   organism g's entries are indptr[g] .. indptr[g + 1]
      indices  int64  [nnz]     column index of each entry (ascending within an organism); on the
                                device u32 (int32 storage) when nnz < 2^32 - 1: read it through
                                column_indices()
      values   uint32 [nnz]     its count

    Codes are 2-bit A0 C1 G2 T3, first base most significant, so code order is the string order
    of the k-mers; for k >= 20 that is the reference's column order (its labels stay the exact
    k-mer text, statistics.py:253-273 and the features2 fixtures), for k <= 19 the reference
    sorts the integer-parsed labels instead (to_frame reproduces it).
    """

    def __init__(self, k, G, lo_code, hi_code, columns, indptr, indices, values, rank=0, world=1):
        self.k, self.G = int(k), int(G)
        self.lo_code, self.hi_code = int(lo_code), int(hi_code)
        self.columns, self.indptr, self.indices, self.values = columns, indptr, indices, values
        self.rank, self.world = rank, world

    @property
    def on_device(self):
        """True when the arrays are device tensors (the GPU path: columns int64 storage of u64,
        values int32 storage of u32); indptr is always a host int64 array."""
        return not isinstance(self.values, np.ndarray)

    @property
    def nnz(self):
        return int(self.values.numel() if self.on_device else self.values.size)

    def host(self):
        """The same shard with numpy arrays (columns uint64, indices int64, values uint32)."""
        if not self.on_device:
            return self
        ix = self.indices.cpu().numpy()
        if ix.dtype == np.int32:   # u32 indices in int32 storage
            ix = ix.view(np.uint32).astype(np.int64)
        return ShardedSparseMatrix(self.k, self.G, self.lo_code, self.hi_code,
                                   self.columns.cpu().numpy().view(np.uint64), np.asarray(self.indptr, np.int64),
                                   ix, self.values.cpu().numpy().view(np.uint32), self.rank, self.world)

    def column_indices(self, a=0, b=None):
        """Entries [a, b)'s column indices as int64 (a device tensor on the GPU path, whose u32
        indices are widened here)."""
        b = self.nnz if b is None else b
        ix = self.indices[a:b]
        if self.on_device:
            import torch
            if ix.dtype == torch.int32:
                return ix.to(torch.int64) & 0xFFFFFFFF
        return ix

    def columns_ascending(self):
        """True iff the columns strictly ascend as unsigned 64-bit codes (on the device the int64
        storage is compared with its sign bit flipped: k = 32 codes use all 64 bits)."""
        if not self.on_device:
            return bool(np.all(self.columns[1:] > self.columns[:-1]))
        import torch
        if self.columns.numel() < 2:
            return True
        c = self.columns ^ torch.iinfo(torch.int64).min
        return bool(torch.all(c[1:] > c[:-1]).item())

    def all_columns_used(self, chunk=1 << 28):
        """True iff every column holds at least one entry (the union has no stray column); chunked
        so that widening u32 indices never needs more than `chunk` int64 entries."""
        if not self.on_device:
            used = np.zeros(self.columns.size, bool)
            used[self.indices] = True
            return bool(used.all())
        import torch
        used = torch.zeros(self.columns.numel(), dtype=torch.uint8, device=self.columns.device)
        for a in range(0, self.nnz, chunk):
            used[self.column_indices(a, min(self.nnz, a + chunk))] = 1
        return bool(torch.all(used == 1).item())

    def __getstate__(self):   # all_gather_object and pickling carry the host form
        return self.host().__dict__

    def dense(self):
        """The shard as a dense [G, ncols] int64 array (small shards only)."""
        h = self.host()
        out = np.zeros((h.G, h.columns.size), np.int64)
        rows = np.repeat(np.arange(h.G), np.diff(h.indptr))
        out[rows, h.indices] = h.values
        return out

    @staticmethod
    def labels(codes, k):
        """The reference's column label of each code: the k-mer's letters; for k <= 19 with the
        leading A's stripped ("A" for A...A), the integer round trip of its k{k}.txt digits
        (statistics.py:157, 248-273)."""
        out = []
        for c in np.asarray(codes, dtype=np.uint64).tolist():
            s = "".join("ACGT"[(c >> (2 * (k - 1 - i))) & 3] for i in range(k))
            out.append((s.lstrip("A") or "A") if k <= 19 else s)
        return out

    @staticmethod
    def to_frame(shards, organisms):
        """Every rank's shard (in rank order, e.g. from torch.distributed.all_gather_object) as
        the reference's DataFrame: organisms x sorted(labels), missing = 0 (small matrices:
        tests and inspection; the distributed matrix itself never materialises densely)."""
        import pandas as pd

        k = shards[0].k
        shards = [s.host() for s in shards]
        cols = np.concatenate([s.columns for s in shards]) if shards else np.zeros(0, np.uint64)
        vals = np.concatenate([s.dense() for s in shards], axis=1) if shards else np.zeros((0, 0), np.int64)
        labels = ShardedSparseMatrix.labels(cols, k)
        order = sorted(range(len(labels)), key=labels.__getitem__)   # features.py:101
        return pd.DataFrame(vals[:, order], index=list(organisms), columns=[labels[i] for i in order])


def _code_splitters(rows, k, world, group):
    """world - 1 code boundaries that cut every rank's entries into ~equal shares: a global
    histogram of the codes' top 16 bits (all-reduced), cut at equal cumulative counts."""
    import torch
    import torch.distributed as dist

    bits = 2 * k
    sh = max(bits - 16, 0)
    nb = 1 << min(bits, 16)
    hist = np.zeros(nb, np.int64)
    for codes, _ in rows:
        if codes.size:
            hist += np.bincount((codes >> np.uint64(sh)).astype(np.int64), minlength=nb)
    t = torch.from_numpy(hist)
    if dist.get_backend(group) != "gloo":
        t = t.cuda()
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return _splitters_from_hist(t.cpu().numpy(), k, world)


def sparse_matrix(genome_files, k, canonical=True, device=None, group=None, rows_fn=None):
    """The organisms x k-mers count matrix for sparse k, column-sharded across the ranks of a
    torch.distributed group: every rank counts its block of genomes
    (sparse_rows: rows sorted by code), the code space is cut into W ranges of ~equal entries,
    and one all-to-all-v (RCCL over xGMI, or gloo) sends each rank the slices of every row that
    fall in its range -- contiguous slices of sorted rows, no scatter.  Returns this rank's
    ShardedSparseMatrix; its columns are the sorted union of the organisms' codes in its range,
    i.e. its share of features.py:96-111's sorted(union of labels).  Without a process group one
    shard holds the whole matrix.  rows_fn(files) -> [(codes uint64 ascending, counts), ...]
    replaces the GPU counter (CPU tests)."""
    import torch
    import torch.distributed as dist

    files = list(genome_files)
    G = len(files)
    if rows_fn is None and 13 <= k <= 32 and G <= SHARD_MAX_ROWS:
        # device-resident: sorted rows, all-to-all, kmh_shard_union_dev (at most SHARD_MAX_ROWS
        # organism rows per shard; larger matrices take the host assembly below)
        return _sparse_matrix_dev(files, k, canonical, device, group)
    if rows_fn is None:
        lo, rows = sparse_rows(files, k, canonical=canonical, device=device, group=group)
    else:
        world0 = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        rank0 = dist.get_rank(group) if world0 > 1 else 0
        lo, hi = shard_bounds(G, world0, rank0)
        rows = rows_fn(files[lo:hi])
    rows = [(np.ascontiguousarray(c, dtype=np.uint64), np.ascontiguousarray(n, dtype=np.uint32)) for c, n in rows]
    if not (dist.is_available() and dist.is_initialized()):
        return _assemble_shard(k, G, 0, 1 << (2 * k), [(lo + i, c, n) for i, (c, n) in enumerate(rows)], 0, 1)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    bounds = _code_splitters(rows, k, world, group)
    # per destination: for each of my genomes, the slice of its sorted row in that range
    # (the last bound, 1 << 2k, may be 1 << 64: every code lies below it, so its cut is len(c))
    inner = np.array(bounds[:-1], dtype=np.uint64)
    cuts = [np.append(np.searchsorted(c, inner, side="left"), c.size) for c, _ in rows]
    send_len = np.array([[int(cut[q + 1] - cut[q]) for cut in cuts] for q in range(world)], np.int64)
    # every rank learns every (source, destination, genome) length: the layout of what it receives
    lens = [None] * world
    dist.all_gather_object(lens, send_len, group=group)
    gpu = dist.get_backend(group) != "gloo"
    codes_out = np.concatenate([rows[i][0][cuts[i][q]:cuts[i][q + 1]] for q in range(world) for i in range(len(rows))]
                               + [np.zeros(0, np.uint64)])
    counts_out = np.concatenate([rows[i][1][cuts[i][q]:cuts[i][q + 1]] for q in range(world) for i in range(len(rows))]
                                + [np.zeros(0, np.uint32)])
    in_splits = [int(send_len[q].sum()) for q in range(world)]
    out_splits = [int(lens[src][rank].sum()) for src in range(world)]

    def a2a(arr, dtype):
        t_in = torch.from_numpy(arr.view(dtype))
        t_out = torch.empty(sum(out_splits), dtype=t_in.dtype)
        if gpu:
            t_in, t_out = t_in.cuda(), t_out.cuda()
        dist.all_to_all_single(t_out, t_in, out_splits, in_splits, group=group)
        return t_out.cpu().numpy()

    rc = a2a(codes_out, np.int64).view(np.uint64)
    rn = a2a(counts_out, np.int32).view(np.uint32)
    # received: source rank by source rank, each source's genomes in order
    parts, pos = [], 0
    for src in range(world):
        glo, _ = shard_bounds(G, world, src)
        for j, n in enumerate(lens[src][rank].tolist()):
            parts.append((glo + j, rc[pos:pos + n], rn[pos:pos + n]))
            pos += n
    return _assemble_shard(k, G, bounds[rank], bounds[rank + 1], parts, rank, world)


def sorted_rows_dev(genome_files, k, canonical=True, device=None, group=None):
    """This rank's block of genomes counted on the GPU with every row in code order
    (kmh_count_sparse_sorted_dev, 13 <= k <= 32), back to back: returns (lo, codes, counts,
    roff) with codes / counts device tensors (int64 / int32 storage of u64 / u32) holding the rows
    back to back, row i = genome lo + i = [roff[i], roff[i + 1]) (roff: host uint64)."""
    import torch
    import torch.distributed as dist

    if not 13 <= k <= 32:
        raise NotImplementedError("sorted device rows need 13 <= k <= 32")
    files = list(genome_files)
    world, rank = 1, 0
    if dist.is_available() and dist.is_initialized():
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_bounds(len(files), world, rank)
    if device is None:
        device = torch.cuda.current_device()
    dev = torch.device("cuda", device)
    if hi == lo:
        return lo, torch.zeros(0, dtype=torch.int64, device=dev), torch.zeros(0, dtype=torch.int32, device=dev), \
            np.zeros(1, np.uint64)
    buf, offsets = pack_genomes(files[lo:hi], k)
    d_seq = torch.from_numpy(buf).to(dev) if buf.size else torch.zeros(16, dtype=torch.uint8, device=dev)
    codes, counts, roff = sorted_rows_from_device(d_seq, offsets, k, canonical)
    return lo, codes, counts, roff


def sorted_rows_from_device(d_seq, offsets, k, canonical=True, timings=None):
    """The sorted rows (as sorted_rows_dev) of genomes already in device memory: d_seq (uint8
    tensor) holds them at offsets (host uint64[n + 1], 16-byte aligned starts).  `timings`: a dict
    that receives the phases' wall times in ms (each phase synchronised; for the bench)."""
    import time
    import torch

    dev = d_seq.device
    tick = [time.perf_counter()]

    def phase(name):
        if timings is not None:
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + (t - tick[0]) * 1e3
            tick[0] = t

    n = len(offsets) - 1
    out_off = _native.sparse_out_offsets(offsets, k)
    cap = max(int(out_off[-1]), 1)
    codes = torch.empty(cap, dtype=torch.int64, device=dev)
    counts = torch.empty(cap, dtype=torch.int32, device=dev)
    nrows = torch.empty(n, dtype=torch.int64, device=dev)
    ndist = torch.empty(n, dtype=torch.int64, device=dev)
    ctx = _native.context(dev.index)
    s = torch.cuda.current_stream(dev).cuda_stream
    phase("alloc_ms")
    ctx.count_sparse_sorted_dev(d_seq.data_ptr(), offsets, k, canonical, codes.data_ptr(), counts.data_ptr(),
                                nrows.data_ptr(), ndist.data_ptr(), s)
    nr, nd = nrows.cpu().numpy(), ndist.cpu().numpy()
    phase("count_ms")
    if not np.array_equal(nr, nd):   # (the library's contract: compact rows)
        raise RuntimeError(f"kmh_count_sparse_sorted_dev: rows of {nr.tolist()} entries for {nd.tolist()} distinct")
    roff = np.zeros(n + 1, np.uint64)
    roff[1:] = np.cumsum(nd)
    return codes, counts, roff   # back to back from entry 0


def _stream(dev):
    import torch

    return torch.cuda.current_stream(dev).cuda_stream


def _rows_cuts(codes, roff, bounds):
    """[n, nb] int64 device tensor: for every sorted row i = codes[roff[i], roff[i + 1]) (host roff)
    the first entry (relative to the row) whose code is >= each bound (kmh_rows_cuts_dev; codes
    compared as u64, so k = 32 needs no sign flip)."""
    import torch

    n, nb = roff.size - 1, len(bounds)
    out = torch.zeros((max(n, 1), max(nb, 1)), dtype=torch.int64, device=codes.device)
    if n and nb and int(roff[-1]) > int(roff[0]):
        _native.context(codes.device.index).rows_cuts_dev(codes.data_ptr(), roff, np.asarray(bounds, np.uint64),
                                                           out.data_ptr(), _stream(codes.device))
    return out[:n, :nb]


def _row_histogram(codes, roff, k, nbits=16):
    """Counts of the rows' codes per top-`nbits`-bit prefix, a device int64 tensor (the rows' cuts at
    every prefix edge, kmh_rows_cuts_dev: binary searches, no pass over the entries)."""
    import torch

    bits = 2 * k
    sh = max(bits - nbits, 0)
    nb = 1 << min(bits, nbits)
    n = roff.size - 1
    dev = codes.device
    if n == 0:
        return torch.zeros(nb, dtype=torch.int64, device=dev)
    cuts = _rows_cuts(codes, roff, [i << sh for i in range(1, nb)])
    lens = torch.from_numpy(np.diff(roff).astype(np.int64)).to(dev)
    full = torch.cat([torch.zeros((n, 1), dtype=torch.int64, device=dev), cuts, lens[:, None]], 1)
    return (full[:, 1:] - full[:, :-1]).sum(0)


def _sparse_matrix_dev(files, k, canonical, device, group):
    """sparse_matrix on the GPU: sorted device rows (sorted_rows_dev), then shard_from_rows."""
    lo, codes, counts, roff = sorted_rows_dev(files, k, canonical=canonical, device=device, group=group)
    held = [codes, counts]
    del codes, counts
    return shard_from_rows(held[0], held[1], roff, len(files), k, group=group, owned=held)


# the exchange of the last shard_from_rows call with W > 1 ranks (bench / tests): wire format, bytes
# this rank sent and received over the all-to-all, and their raw (12 B per entry) equivalent
LAST_EXCHANGE = None
WIRE_RECORD_ENTRIES = 1024        # entries per record of the compact wire (kmh_wire.hip)
SHARD_MAX_ROWS = 4096             # kmh_shard_union_dev's limit on the organism rows of one shard


def shard_plan(codes, roff, bounds, rank):
    """The slices this rank's sorted rows send to every rank's code range [bounds[q], bounds[q + 1]):
    returns (send_len [n, W] int64: entries of row j in range q, starts [n, W] int64: their first
    entry in `codes`).  One device cuts call and one host copy."""
    n, W = roff.size - 1, len(bounds) - 1
    lens = np.diff(roff).astype(np.int64)
    cuts = _rows_cuts(codes, roff, bounds[1:-1]).cpu().numpy() if n else np.zeros((0, W - 1), np.int64)
    full = np.concatenate([np.zeros((n, 1), np.int64), cuts, lens[:, None]], 1)
    return np.diff(full, axis=1), roff[:-1].astype(np.int64)[:, None] + full[:, :-1]


def _a2a(out, inp, out_splits, in_splits, gloo, group):
    import torch
    import torch.distributed as dist

    if gloo:   # gloo exchanges host tensors
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(ho, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(ho)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


def shard_from_rows(codes, counts, roff, G, k, group=None, wire="auto", timings=None, owned=None):
    """This rank's ShardedSparseMatrix from its sorted device rows (genomes shard_bounds(G, W,
    rank), row i = codes / counts [roff[i], roff[i + 1])).  With W > 1 ranks:

      1. the code space is cut into W ranges of ~equal entries: an all-reduced histogram of the
         codes' top 16 bits, from the rows' cuts at every prefix edge (kmh_rows_cuts_dev);
      2. the rows' cuts at the W - 1 range bounds give every (row, rank) slice (one host copy) and
         one all_gather tells every rank what it receives;
      3. the slices for the other ranks are packed in the compact wire format (kmh_wire_encode_dev,
         ~2.2 B per entry against 12; wire="raw" sends u64 codes + u32 counts, and "auto" falls back
         to raw when the packed bytes would be larger, e.g. k = 32 codes with 40-bit gaps), sent by
         ONE all_to_all_single (RCCL over xGMI, or gloo), and unpacked straight into the shard's row
         layout (kmh_wire_decode_dev); the rank's own slices are device copies;
      4. kmh_shard_union(_u32)_dev builds the columns (the sorted union: features.py:96-111) and
         the CSR indices, u32 whenever the shard holds fewer than 2^32 - 1 entries.

    Every array stays in device memory.  `timings` (a dict) receives per-phase wall ms (each phase
    synchronised; bench).  `owned`: a list holding the caller's only references to codes and counts;
    it is cleared once the rows have been sent, so their memory (12 B per entry) is free before the
    receive side and the union allocate theirs (at N = 8, 48 GB per rank)."""
    import time
    import torch
    import torch.distributed as dist

    global LAST_EXCHANGE
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    dev = codes.device
    n = roff.size - 1
    ctx = _native.context(dev.index)
    s = _stream(dev)
    tick = [time.perf_counter()]

    def phase(name):
        if timings is not None:
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + (t - tick[0]) * 1e3
            tick[0] = t

    if world == 1:   # one shard: every genome's row, the whole code space
        rc, rn, indptr, lo_code, hi_code = codes, counts, roff.astype(np.int64), 0, 1 << (2 * k)
    else:
        gloo = dist.get_backend(group) == "gloo"
        hist = _row_histogram(codes, roff, k)
        if gloo:
            hist = hist.cpu()
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
        bounds = _splitters_from_hist(hist.cpu().numpy(), k, world)
        send_len, starts = shard_plan(codes, roff, bounds, rank)
        phase("plan_ms")
        B = block_rows(G, world)
        others = [q for q in range(world) if q != rank]
        sl_start = np.array([starts[j, q] for q in others for j in range(n)], np.uint64)
        sl_n = np.array([send_len[j, q] for q in others for j in range(n)], np.uint64)
        raw_bytes = int(sl_n.sum()) * 12
        mode = wire
        sl_bytes = sl_n * np.uint64(12)
        if wire in ("auto", "compact"):
            sl_bytes = ctx.wire_size_dev(codes.data_ptr(), counts.data_ptr(), sl_start, sl_n, s) if sl_n.size else sl_n
            if wire == "auto":   # every rank must choose the same format
                t = torch.tensor([int(sl_bytes.sum()), raw_bytes], dtype=torch.int64)
                if not gloo:
                    t = t.to(dev)
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
                t = t.cpu()
                mode = "compact" if int(t[0]) < int(t[1]) else "raw"
            if mode == "raw":
                sl_bytes = sl_n * np.uint64(12)
        # every rank learns (entries, bytes) of every (source, genome index, destination) slice
        mine = np.zeros((B, world, 2), np.int64)
        mine[:n, :, 0] = send_len
        for i, q in enumerate(others):
            mine[:n, q, 1] = sl_bytes[i * n:(i + 1) * n].astype(np.int64)
        lt = torch.from_numpy(mine) if gloo else torch.from_numpy(mine).to(dev)
        parts = [torch.zeros_like(lt) for _ in range(world)]
        dist.all_gather(parts, lt, group=group)
        lens = np.stack([t.cpu().numpy() for t in parts])   # lens[src, j, dst, (entries, bytes)]
        # receive layout: genome-major (= source-major: rank src holds genomes shard_bounds(G, W, src))
        gl = np.zeros(G, np.int64)
        gsrc = []
        for src in range(world):
            glo, ghi = shard_bounds(G, world, src)
            gl[glo:ghi] = lens[src, :ghi - glo, rank, 0]
            gsrc.append((glo, ghi))
        indptr = np.zeros(G + 1, np.int64)
        np.cumsum(gl, out=indptr[1:])
        total = int(indptr[-1])
        phase("sizes_ms")
        rc = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
        rn = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        lo_g = gsrc[rank][0]
        if mode == "raw":   # u64 codes + u32 counts, the rank's own slices included
            sel = [(int(starts[j, q]), int(send_len[j, q])) for q in range(world) for j in range(n)]
            in_splits = [int(send_len[:, q].sum()) for q in range(world)]
            out_splits = [int(lens[src, :, rank, 0].sum()) for src in range(world)]
            for src_t, dst_t in ((codes, rc), (counts, rn)):
                inp = torch.cat([src_t[a:a + m] for a, m in sel] + [src_t[:0]])
                _a2a(dst_t[:total], inp, out_splits, in_splits, gloo, group)
                del inp
            sent, received = raw_bytes, int(sum(out_splits[q] for q in others)) * 12
            if owned is not None:
                owned.clear()
            phase("exchange_ms")
        else:
            for j in range(n):   # the rank's own slices: device copies into place
                a, m, d = int(starts[j, rank]), int(send_len[j, rank]), int(indptr[lo_g + j])
                if m:
                    rc[d:d + m].copy_(codes[a:a + m])
                    rn[d:d + m].copy_(counts[a:a + m])
            nbytes = int(sl_bytes.sum())
            send = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
            if sl_n.size:
                ctx.wire_encode_dev(codes.data_ptr(), counts.data_ptr(), sl_start, sl_n, send.data_ptr(), nbytes, s)
            if owned is not None:   # the rows are sent: free them before the receive buffers
                owned.clear()
                del codes, counts
                codes = counts = None
            phase("encode_ms")
            in_splits = [0 if q == rank else int(sl_bytes[others.index(q) * n:(others.index(q) + 1) * n].sum())
                         for q in range(world)]
            out_splits = [0 if src == rank else int(lens[src, :, rank, 1].sum()) for src in range(world)]
            recv = torch.empty(max(sum(out_splits), 16), dtype=torch.uint8, device=dev)
            _a2a(recv[:sum(out_splits)], send[:nbytes], out_splits, in_splits, gloo, group)
            del send
            phase("exchange_ms")
            rs_n, rs_b, rs_d = [], [], []
            for src in others:
                glo, ghi = gsrc[src]
                for j in range(ghi - glo):
                    rs_n.append(lens[src, j, rank, 0])
                    rs_b.append(lens[src, j, rank, 1])
                    rs_d.append(indptr[glo + j])
            if rs_n:
                ctx.wire_decode_dev(recv.data_ptr(), sum(out_splits), np.array(rs_n, np.uint64),
                                    np.array(rs_b, np.uint64), np.array(rs_d, np.uint64), rc.data_ptr(),
                                    rn.data_ptr(), s)
            del recv
            sent, received = nbytes, sum(out_splits)
            phase("decode_ms")
        LAST_EXCHANGE = {"wire": mode, "sent_bytes": int(sent), "received_bytes": int(received),
                         "raw_sent_bytes": raw_bytes,
                         "raw_received_bytes": int(sum(lens[src, :, rank, 0].sum() for src in others)) * 12,
                         "entries_in": int(np.diff(roff).sum()) if n else 0, "entries_out": total}
        del codes, counts
        lo_code, hi_code = bounds[rank], bounds[rank + 1]
    total = int(indptr[-1])
    if total and indptr.size - 1 > SHARD_MAX_ROWS:
        raise NotImplementedError(f"kmh_shard_union_dev holds at most {SHARD_MAX_ROWS} organism rows per shard "
                                  f"(got {indptr.size - 1}); sparse_matrix routes such matrices to the host path")
    idx32 = total < 0xFFFFFFFF
    columns = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    indices = torch.empty(max(total, 1), dtype=torch.int32 if idx32 else torch.int64, device=dev)
    ncols = 0
    if total and hi_code > lo_code:
        ncols = ctx.shard_union_dev(rc.data_ptr(), indptr.astype(np.uint64), lo_code, hi_code - 1, columns.data_ptr(),
                                    indices.data_ptr(), s, idx32=idx32)
    elif total:
        raise RuntimeError(f"rank {rank} received {total} entries for the empty code range [{lo_code}, {hi_code})")
    phase("union_ms")
    return ShardedSparseMatrix(k, G, lo_code, hi_code, columns[:ncols], indptr, indices[:total], rn[:total],
                               rank, world)


def shard_check(m, windows_total, group=None):
    """Global checks of a column-sharded matrix (every rank calls it; returns (ok, summary)): within
    the rank, columns strictly ascending and every column used; across ranks, sum(values) over all
    shards = windows_total (every window of every genome counted exactly once: a slice lost or sent
    twice by the exchange changes it), sum(nnz) consistent with it, and rank q's last column below
    rank q + 1's first.  Returns the all-reduced summary (nnz, values, columns)."""
    import torch
    import torch.distributed as dist

    cols = m.columns
    dev = cols.device
    ok = m.columns_ascending() and m.all_columns_used()
    vsum = int((m.values.to(torch.int64) & 0xFFFFFFFF).sum().item()) if m.nnz else 0
    # (k = 32 codes use all 64 bits: as int64 they would not order; compare the unsigned values)
    first = int(cols[0].item()) & 0xFFFFFFFFFFFFFFFF if cols.numel() else None
    last = int(cols[-1].item()) & 0xFFFFFFFFFFFFFFFF if cols.numel() else None
    ok = ok and all(m.lo_code <= c < m.hi_code for c in (first, last) if c is not None)
    world = m.world
    if world > 1:
        gloo = dist.get_backend(group) == "gloo"
        t = torch.tensor([m.nnz, vsum, int(cols.numel()), 0 if ok else 1], dtype=torch.int64)
        t = t if gloo else t.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        nnz, vsum, ncols, bad = (int(x) for x in t.cpu().tolist())
        ends = [None] * world
        dist.all_gather_object(ends, (m.rank, first, last), group=group)
        ok = bad == 0
        prev = None
        for _, f, l in sorted(ends):
            if f is None:
                continue
            ok = ok and (prev is None or prev < f)
            prev = l
    else:
        nnz, ncols = m.nnz, int(cols.numel())
    ok = ok and vsum == windows_total and ncols <= nnz <= vsum
    return ok, {"nnz": nnz, "values": vsum, "columns": ncols}


def _splitters_from_hist(hist, k, world):
    """world - 1 code boundaries cutting a histogram of the codes' top bits (all ranks' rows)
    into ~equal shares (as _code_splitters)."""
    bits = 2 * k
    sh = max(bits - 16, 0)
    nb = 1 << min(bits, 16)
    cum = np.cumsum(hist)
    total = int(cum[-1]) if cum.size else 0
    # bucket indices stay unshifted (monotone, <= nb) until the end; the last bound is the
    # code space's end, 1 << 64 at k = 32 (a Python int: never converted to uint64)
    # inner bounds at most (nb - 1) << sh, so every one stays below the code space's end (< 2^64 at
    # k = 32: a bound of 1 << 64 would not survive the uint64 conversions of the exchange); ranks
    # past a bound in the last bucket get an empty range
    idx = [0]
    for q in range(1, world):
        b = int(np.searchsorted(cum, total * q / world, side="left")) + 1 if total else (nb * q) // world
        idx.append(max(idx[-1], min(b, nb - 1)))
    return [i << sh for i in idx] + [1 << bits]


def _assemble_shard(k, G, lo_code, hi_code, parts, rank, world):
    """CSR of one column shard from (genome, sorted codes, counts) pieces."""
    per = [None] * G
    for g, c, n in parts:
        per[g] = (c, n)
    per = [p if p is not None else (np.zeros(0, np.uint64), np.zeros(0, np.uint32)) for p in per]
    allc = np.concatenate([c for c, _ in per]) if per else np.zeros(0, np.uint64)
    columns = np.unique(allc)
    indptr = np.zeros(G + 1, np.int64)
    np.cumsum([c.size for c, _ in per], out=indptr[1:])
    indices = np.searchsorted(columns, allc).astype(np.int64)
    values = np.concatenate([n for _, n in per]) if per else np.zeros(0, np.uint32)
    return ShardedSparseMatrix(k, G, lo_code, hi_code, columns, indptr, indices, values, rank, world)
