"""Benchmark: bases/s counted into the genomes x k-mers count matrix on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--k 12] [--genomes 64]
                  [--genome-len 100000000] [--assemble auto|allgather|none]

Workload (BASELINE.json configs): N = 1 is config 3 -- 64 synthetic 100 Mbp genomes,
k = 12, dense 4^12 histogram per genome on one MI355X.  N > 1 is config 4 -- the same 64
genomes sharded in contiguous blocks of 64/N per GPU (one process per GPU, launched by
torch.distributed.run) with an RCCL all-gather that assembles the [64, 4^12] u32 matrix on
every rank inside each step (sent as saturating u4 rows + an exact escape list, step i's
all-gather overlapped with step i+1's count; --assemble u8 / u32 send u8 / plain rows).  A step is one pass of the count path over every genome
(plus the all-gather for N > 1); the genomes are generated on the device before timing,
so inputs are resident in HBM when the timed region starts.

Printed by rank 0: one JSON line with the driver's fields plus
  roofline      the dominant kernel: algorithmic bytes per launch / mean launch time
                (HIP events on the launch stream) against 8 TB/s;
  step_roofline the whole step per GPU: (its genomes' bases * 1 B + the count rows it ends up
                holding * 4 B) / step time / 8 TB/s; reads_only_frac = bases / step time / 8 TB/s;
  cpu_baseline  the reference's algorithm (oracle/kmers.py, the same pure-Python window
                loop as generate.py:49-58) timed on one host core over a bounded sample.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "kmer-ml_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kmerml import _native  # noqa: E402

METRIC = "bases/s counted into k-mer feature matrix (1/2/4/8 GPU) + % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
XGMI_LINK_GBS = 153.0          # one xGMI link per direction; 7 links per MI355X
SEED_BASE = 0x6B6D65724D4C0000


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--min-warmup-ms", type=float, default=60.0,
                   help="dense workload: after the --warmup steps, more untimed steps until the warm-up "
                        "has run this long (the same number on every rank).  The GPU takes ~30-50 ms "
                        "of load to reach its steady rate: one N = 8 rank (1.2 ms steps) measured "
                        "1.20-1.21 ms per step after 3 warm-up steps and 1.13-1.14 after 30 "
                        "(profiles/r05/r05ae, r05af); config 3's 8 ms steps are steady after 3.  0 = off; "
                        "the line reports the steps run as warmup_steps_run")
    p.add_argument("--workload", choices=["dense", "sparse"], default="dense",
                   help="dense = configs 3/4 (default); sparse = config 5 (k = 21 canonical, "
                        "250 Mbp genomes, 16 per GPU, no collective)")
    p.add_argument("--k", type=int, default=None, help="default 12 (dense) / 21 (sparse)")
    p.add_argument("--genomes", type=int, default=None,
                   help="total genomes over all ranks (default 64 dense / 16 per GPU sparse)")
    p.add_argument("--genome-len", type=int, default=None, help="default 100 Mbp dense / 250 Mbp sparse")
    p.add_argument("--forward", action="store_true", help="sparse: forward-strand codes instead of canonical")
    p.add_argument("--assemble", choices=["auto", "u4", "u4-dense", "u8", "u32", "none"], default="auto",
                   help="N > 1 matrix assembly.  u4 (default): saturating 4-bit rows + exact escape "
                        "list on the wire, all-gather overlapped with the next step's count, and the "
                        "assembled matrix kept in that exact compact form on every rank (rows widened "
                        "on access, kmerml.kmers.matrix.AssembledMatrix); u4-dense / u8: the same "
                        "wire, every gathered row widened to the u32 matrix on every rank each step; "
                        "u32 = plain all-gather of the u32 rows after each count")
    p.add_argument("--separate-encode", action="store_true",
                   help="compact u4 assembly: count, then encode in a second pass (A/B of the fused "
                        "kmh_count_dense_u4_dev)")
    p.add_argument("--no-matrix", action="store_true",
                   help="--workload sparse (and the config-5 object): skip the column-sharded matrix leg")
    p.add_argument("--no-config5", action="store_true",
                   help="dense N = 1: skip the config-5 measurement (16 x 250 Mbp, k = 21 canonical, "
                        "3 timed steps) that the default run appends to its JSON line as \"config5\"")
    p.add_argument("--no-e2e", action="store_true",
                   help="dense N = 1: skip the drop-in end-to-end leg (the reference CLI's call pattern on "
                        "synthetic FASTA files, per-stage clocks) that the default run appends as \"e2e\"")
    p.add_argument("--simulate-ranks", type=int, default=0,
                   help="one process on one GPU doing what ONE rank of N does per step: dense = config 4 "
                        "(count G/N genomes, encode u4, and the all-gather's writes modelled as N - 1 "
                        "device copies of the slot; no xGMI); sparse = config 5's matrix (--genomes per "
                        "rank, the other ranks' slices of its code range really counted and packed, "
                        "unpacked and unioned at R = N x genomes rows): a projection, labelled as such")
    p.add_argument("--matrix-wire", choices=["auto", "compact", "raw"], default="auto",
                   help="config-5 matrix at N > 1: the all-to-all's wire (auto = compact gaps unless raw u64 + "
                        "u32 is smaller, e.g. small genomes or k = 32; kmerml.kmers.matrix.shard_from_rows)")
    p.add_argument("--config5-genomes-per-rank", type=int, default=16,
                   help="the config-5 object of the dense line: genomes per rank (config 5: 128 / 8 = 16)")
    p.add_argument("--config5-genome-len", type=int, default=250_000_000,
                   help="the config-5 object of the dense line: genome length (config 5: 250 Mbp; smaller "
                        "only for rehearsals, which the object then labels)")
    p.add_argument("--sim-copy", choices=("torch", "none"), default="torch",
                   help="--simulate-ranks: model the all-gather's writes by device copies (torch), or "
                        "leave them out (none: isolates the copies' contention with the count)")
    p.add_argument("--cpu-sample", type=int, default=8_000_000,
                   help="bases of genome 0 timed with the reference-algorithm CPU loop (0 = skip)")
    p.add_argument("--kernel-events", choices=["roofline", "all"], default="roofline",
                   help="HIP event pairs around the kernels the roofline names only (default), or all")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="experiments: no per-kernel HIP events in the timed region (roofline = null)")
    p.add_argument("--pmc-summary", default=os.path.join(HERE, "profiles", "pmc_traffic.json"),
                   help="rocprofv3 FETCH_SIZE / WRITE_SIZE summary (profiles/pmc_summary.py); its "
                        "figure is printed only if it was measured on this library's build id")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="process-group backend (gloo + --single-device: multi-rank logic check on one GPU)")
    p.add_argument("--check-dir", default=None,
                   help="after timing, verify the assembled matrix on every rank against every rank's "
                        "own count rows (row signatures), and have rank 0 save the assembled rows of "
                        "genomes 0 and G-1 there as .npy (tests compare them with the oracle)")
    p.add_argument("--single-device", action="store_true",
                   help="map every rank to cuda:0 (validation only; never used for reported numbers)")
    a = p.parse_args()
    dense = a.workload == "dense"
    a.k = a.k if a.k is not None else (12 if dense else 21)
    a.genome_len = a.genome_len if a.genome_len is not None else (100_000_000 if dense else 250_000_000)
    if a.genomes is None:
        a.genomes = 64 if dense else 16 * int(os.environ.get("WORLD_SIZE", "1"))
    return a


CONFIG5_CPU_SAMPLE = 6_000_000    # ~5 s of the k = 21 loop on one EPYC 9575F core + ~10 s of its writer


def cpu_baseline(sample, k, strand=None):
    """Time the reference's per-window loop (oracle restatement, forward strand: the
    reference has no canonical mode) on one core."""
    sys.path.insert(0, HERE)
    from oracle import kmers as okmers
    from oracle import synth as osynth
    import tempfile
    seq = osynth.synth_bases(sample, osynth.genome_seed(0)).tobytes().decode()
    t0 = time.perf_counter()
    table = okmers.count_sequence(seq, k)
    dt = time.perf_counter() - t0
    assert sum(table.values()) == sample - k + 1
    # the save phase (generate.py:68-91, compress=False as the CLI's default) on the same table:
    # SURVEY 8(d) times it separately because it scales with the distinct k-mers, not the bases
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, f"k{k}.txt")
        t1 = time.perf_counter()
        okmers.save_kmers(table, path)
        ds = time.perf_counter() - t1
        save_bytes = os.path.getsize(path)
    note = (" (forward strand: the reference counts no canonical k-mers, so this is its loop on "
            "the config's genomes, not a canonical count)") if strand == "forward" else ""
    return {"value": sample / dt, "unit": "bases/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} bases of synthetic genome 0, k={k}: the count loop of "
                      f"generate.py:49-58 restated in pure Python (oracle/kmers.py), "
                      f"{dt:.2f} s on one core{note}; then its k{k}.txt writer (generate.py:68-91, "
                      f"oracle/kmers.py save_kmers) over the {len(table)} distinct k-mers, {ds:.2f} s",
            "k": k, "seconds": dt, "save_seconds": ds, "save_lines": len(table), "save_bytes": save_bytes,
            "value_e2e": sample / (dt + ds),
            "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count()}


def cpu_threads_baseline(k, bases_per_thread=25_000_000, threads=16):
    """A stronger CPU reference point beside the 1-core loop: the C restatement of the
    counting rule (oracle/kmer_oracle.c, dense 4^k table, one private table per thread) on
    `threads` host threads, each counting its own synthetic genome (ctypes releases the GIL).
    Not the reference's code path -- reported as kind "port"."""
    sys.path.insert(0, HERE)
    from concurrent.futures import ThreadPoolExecutor
    from oracle import corac
    from oracle import synth as osynth
    if k > 12:
        return None
    seqs = [corac.synth(bases_per_thread, osynth.genome_seed(g)) for g in range(threads)]
    corac.count_dense(seqs[0][:1000], k)       # load the library outside the timed region
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        tables = list(ex.map(lambda q: corac.count_dense(q, k), seqs))
    dt = time.perf_counter() - t0
    assert all(int(t.sum()) == bases_per_thread - k + 1 for t in tables)
    return {"value": threads * bases_per_thread / dt, "unit": "bases/s", "cores": threads, "kind": "port",
            "sample": f"{threads} synthetic genomes x {bases_per_thread} bases, k={k}: C restatement of "
                      f"generate.py:49-58 (oracle/kmer_oracle.c) on {threads} threads, {dt:.2f} s"}


def _ref_loop_genome(args):
    """One process of cpu_procs_baseline: the restated reference loop over its own genome."""
    g, n, k = args
    from oracle import kmers as okmers
    from oracle import synth as osynth
    seq = osynth.synth_bases(n, osynth.genome_seed(g)).tobytes().decode()
    t0 = time.perf_counter()
    table = okmers.count_sequence(seq, k)
    dt = time.perf_counter() - t0
    assert sum(table.values()) == n - k + 1
    return dt


def cpu_procs_baseline(k, bases_per_proc=4_000_000, procs=None):
    """SURVEY.md 8(d) "ref-CPU x P": the reference's per-window Python loop (oracle/kmers.py
    restates generate.py:49-58) with one genome per process on P host cores.  The reference
    itself is serial (scripts/extract_kmers.py:58-61 loops over genomes), so this is the best
    its algorithm does on this host without changing it.  P = the cores this process may use,
    at most 16 (one GPU's share of the box).  Forked before the GPU is touched."""
    import multiprocessing as mp
    sys.path.insert(0, HERE)
    if procs is None:
        procs = max(1, min(16, len(os.sched_getaffinity(0))))
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(procs) as pool:
        per = pool.map(_ref_loop_genome, [(g, bases_per_proc, k) for g in range(procs)])
    dt = time.perf_counter() - t0
    # rate over the count loops, which run concurrently (the slowest sets it); the wall time
    # also holds pool start-up and each process generating its genome
    return {"value": procs * bases_per_proc / max(per), "unit": "bases/s", "cores": procs, "kind": "port",
            "sample": f"{procs} synthetic genomes x {bases_per_proc} bases, k={k}, one genome per process: "
                      f"the count loop of generate.py:49-58 restated in pure Python (oracle/kmers.py), "
                      f"slowest process {max(per):.2f} s ({dt:.2f} s wall with start-up)"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def load_traffic(path, config_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this command.

    Returns (entry, note).  An entry measured on another build of the library (its
    "build_id" differs from kmh_build_id() of the loaded one) is stale and not returned.
    """
    from kmerml import _native

    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary"
    entry = d.get(config_key)
    if not isinstance(entry, dict):
        return None, f"no PMC entry {config_key}"
    lib_id = _native.build_id()
    if entry.get("build_id") != lib_id:
        return None, f"stale PMC entry (build {entry.get('build_id')}, library {lib_id})"
    return entry, f"rocprofv3 FETCH_SIZE/WRITE_SIZE passes on build {lib_id} ({entry.get('source', '')})"


def row_signatures(rows):
    """[n, 2] int64 per row: the sum and sum(value * (column + 1)) (int64, wrapping), one row
    at a time (a whole-matrix int64 temporary would be 8 x its size)."""
    n, bins = rows.shape
    w = torch.arange(1, bins + 1, dtype=torch.int64, device=rows.device)
    out = torch.empty((n, 2), dtype=torch.int64, device=rows.device)
    for i in range(n):
        r = rows[i].to(torch.int64) & 0xFFFFFFFF
        out[i, 0] = r.sum()
        out[i, 1] = (r * w).sum()
    return out.cpu()


def check_assembly(full, own, B, G, world, rank, k, check_dir):
    """Every rank's assembled matrix against every rank's own count rows: rank q's block of
    `full` (rows q*B ..) must have the signatures rank q computed from the rows it counted
    (which, at N > 1, every other rank only sees after encode -> all-gather -> decode).  Rank 0
    also saves the assembled rows of genomes 0 and G - 1 for an oracle comparison."""
    mine = row_signatures(own)
    if world > 1:
        sigs = [None] * world
        dist.all_gather_object(sigs, mine)
    else:
        sigs = [mine]
    ok = True
    for q in range(world):
        lo, hi = (G * q) // world, (G * (q + 1)) // world
        got = row_signatures(full[q * B:q * B + (hi - lo)])
        ok = ok and torch.equal(got, sigs[q])
    if rank == 0:
        os.makedirs(check_dir, exist_ok=True)
        last_q = world - 1
        last_row = last_q * B + (G - 1 - (G * last_q) // world)
        np.save(os.path.join(check_dir, "row_first.npy"), full[0].cpu().numpy().view(np.uint32))
        np.save(os.path.join(check_dir, "row_last.npy"), full[last_row].cpu().numpy().view(np.uint32))
    return bool(ok)


def allgather_report(mode, world, B, bins, gather_ms, gloo, scope):
    """the matrix assembly's all-gather on its own -- time per step (mean over the
    timed steps, max over ranks; RCCL: HIP events on the comm stream, which include waiting for
    the slowest peer), bytes each rank receives, and that rate against the xGMI links: all 7 of
    an MI355X (7 x 153 GB/s, SURVEY's figure) and the N - 1 links that reach the other ranks."""
    if mode == "none" or gather_ms is None:
        return None
    per_rank = {"u32": B * bins * 4}.get(mode, scope.get("P"))
    recv_bytes = (world - 1) * per_rank
    gbs = recv_bytes / (gather_ms * 1e-3) / 1e9 if gather_ms > 0 else None
    return {"allgather_ms": round(gather_ms, 4), "wire": mode, "slot_bytes": per_rank,
            "received_bytes_per_rank": recv_bytes,
            "received_GBs_per_gpu": round(gbs, 1) if gbs is not None else None,
            "frac_of_7_links": round(gbs / (7 * XGMI_LINK_GBS), 4) if gbs is not None else None,
            "frac_of_peer_links": (round(gbs / ((world - 1) * XGMI_LINK_GBS), 4)
                                   if gbs is not None and world > 1 else None),
            "timing": "gloo host-staged, wall clock (validation only)" if gloo else
                      "HIP events around the RCCL all-gather on its own stream (includes peer skew)"}


def workload_name(G, L, k, world, single_device, backend):
    """BASELINE.json config label -- only for the configs' own sizes on real devices; anything
    else (smaller genomes, ranks sharing one GPU) is labelled a rehearsal."""
    shape = f"{G} synthetic {L / 1e6:g} Mbp genomes, k={k} dense 4^{k} count matrix"
    if world > 1:
        shape += f", sharded {G}/{world} per rank + {backend} all-gather"
    real = G == 64 and L == 100_000_000 and k == 12 and not single_device
    if single_device:
        return f"rehearsal ({world} ranks sharing cuda:0, not a config-4 measurement): {shape}"
    if not real:
        return f"non-baseline size: {shape}"
    return f"config{3 if world == 1 else 4}: {shape}"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    # CPU baselines first (rank 0, N = 1 only), before the GPU is touched (the process pool
    # forks) and so that they never overlap GPU timing.
    cpu = cpu_mt = cpu_p = cpu5 = None
    if a.workload == "dense" and rank == 0 and world == 1 and a.cpu_sample > 0:
        cpu = cpu_baseline(a.cpu_sample, a.k)
        cpu_p = cpu_procs_baseline(a.k)
        cpu_mt = cpu_threads_baseline(a.k)
        if not a.no_config5:
            cpu5 = cpu_baseline(CONFIG5_CPU_SAMPLE, 21, strand="forward")
    dev_index = 0 if a.single_device else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    # A process group for N > 1, or when torch.distributed.run launched a single rank with an
    # explicit assembly mode (exercises the RCCL code path on one GPU).
    use_dist = world > 1 or (a.assemble in ("u4", "u4-dense", "u8", "u32") and "RANK" in os.environ)
    if use_dist:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)   # RCCL over xGMI
        else:
            dist.init_process_group("gloo")
    k, G, L = a.k, a.genomes, a.genome_len
    if a.workload == "sparse":
        if a.simulate_ranks > 1 and world == 1:
            return run_sparse_sim(a, dev, dev_index)
        return run_sparse(a, world, rank, dev, dev_index)
    sim = a.simulate_ranks if world == 1 and a.simulate_ranks > 1 else 0
    span = sim or world                       # ranks the genomes are sharded over
    lo, hi = (G * rank) // span, (G * (rank + 1)) // span
    g_local = hi - lo
    B = -(-G // span)
    mode = ("u4" if world > 1 else "none") if a.assemble == "auto" else a.assemble
    if sim:
        mode = "u4"
    assemble = mode != "none"
    bins = 1 << (2 * k)

    ctx = _native.context(dev_index)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    stride = (L + 15) // 16 * 16   # genome starts 16-byte aligned; any gap is 'N' (not a base)
    d_seq = torch.empty(max(g_local, 1) * stride, dtype=torch.uint8, device=dev)
    if stride != L:
        d_seq.fill_(ord("N"))
    if g_local:
        ctx.synth_dev(d_seq.data_ptr(), L, stride, g_local, SEED_BASE + lo, s)
    offsets = np.arange(g_local + 1, dtype=np.uint64) * np.uint64(stride)
    gloo = a.backend == "gloo"
    full = torch.empty((world * B, bins), dtype=torch.int32, device=dev) if mode == "u32" else None
    t_count = []
    t_gather = []          # per timed step: (start, end) events on the comm stream, or gloo wall ms
    comm = torch.cuda.Stream(dev) if use_dist and not gloo else None

    def gather(recv_t, send_t, record):
        """All-gather send_t of every rank into recv_t (SURVEY 8(e)'s one exchange step).  RCCL:
        issued from the `comm` stream after the count that wrote send_t, with a HIP event pair
        around it on that stream (the time includes waiting for the slowest peer); returns the
        event the consumer waits for, so step i+1's count overlaps it.  gloo: host-staged and
        synchronous (validation only), timed by the wall clock."""
        if gloo:
            t0 = time.perf_counter()
            host = torch.empty(tuple(recv_t.shape), dtype=recv_t.dtype)
            dist.all_gather_into_tensor(host, send_t.cpu())
            recv_t.copy_(host)
            if record:
                t_gather.append((time.perf_counter() - t0) * 1e3)
            return None
        comm.wait_stream(stream)
        with torch.cuda.stream(comm):
            e0 = torch.cuda.Event(enable_timing=True) if record else None
            if record:
                e0.record(comm)
            dist.all_gather_into_tensor(recv_t, send_t)
            done = torch.cuda.Event(enable_timing=record)
            done.record(comm)
        if record:
            t_gather.append((e0, done))
        return done

    def count_into(buf, record, u4=None):
        e0 = torch.cuda.Event(enable_timing=True) if record else None
        e1 = torch.cuda.Event(enable_timing=True) if record else None
        if record:
            e0.record(stream)
        if g_local and u4 is not None:   # buf is scratch here (kmh_count_dense_u4only_dev)
            ctx.count_dense_u4_dev(d_seq.data_ptr(), offsets, k, buf.data_ptr(), *u4, s, rows=False)
        elif g_local:
            ctx.count_dense_dev(d_seq.data_ptr(), offsets, k, buf.data_ptr(), s)
        if record:
            e1.record(stream)
            t_count.append((e0, e1))

    if mode == "u4":
        # Compact assembly (the N > 1 default): step i counts this rank's rows into
        # `local`, encodes them into send[i % 2] (u4 + exact escapes) and all-gathers the slots
        # into recv[i % 2] on RCCL's stream, overlapped with step i+1's count; the assembled
        # matrix of step i IS recv[i % 2] (every rank's slot; AssembledMatrix widens rows on
        # access).  Step i+2 waits for step i's all-gather before it reuses the buffers.
        from kmerml.kmers.matrix import AssembledMatrix, slot_layout_u4
        cap, P = slot_layout_u4(B, bins)
        payload = B * bins // 2
        local = torch.zeros((B, bins), dtype=torch.int32, device=dev)
        locals_ = [local]
        recv = [torch.zeros(span * P, dtype=torch.uint8, device=dev) for _ in range(2)]
        # in-place all-gather (RCCL's in-place form, sendbuff = recvbuff + rank * count): the
        # rank's own slot of recv IS its send buffer, written once by the count, never copied
        send = [r[rank * P:(rank + 1) * P] for r in recv]
        inflight = [None, None]
        side = torch.cuda.Stream(dev) if sim else None

        def step(i, record=False):
            b = i % 2
            if inflight[b] is not None:      # step i-2's all-gather (send[b] -> recv[b])
                w = inflight[b]
                stream.wait_event(w) if isinstance(w, torch.cuda.Event) else w.wait()
                inflight[b] = None
            sb = send[b]
            if a.separate_encode or not g_local:
                count_into(local, record)
                ctx.rows_encode_u4(local.data_ptr(), B, bins, sb.data_ptr(), sb[payload + 16:].data_ptr(),
                                   cap, sb[payload:].data_ptr(), s)
            else:   # count + u4 encode in one pass (kmh_count_dense_u4_dev)
                count_into(local, record, u4=(sb.data_ptr(), sb[payload + 16:].data_ptr(), cap,
                                              sb[payload:].data_ptr()))
            if sim:   # the gather's HBM side: every other slot of recv written (from this rank's)
                side.wait_stream(stream)
                with torch.cuda.stream(side):
                    for q in range(1, span if a.sim_copy == "torch" else 1):
                        recv[b][q * P:(q + 1) * P].copy_(sb)
                    ev = torch.cuda.Event()
                    ev.record(side)
                inflight[b] = ev
            else:
                inflight[b] = gather(recv[b], sb, record)

        def drain():
            for b in range(2):
                if inflight[b] is not None:
                    w = inflight[b]
                    stream.wait_event(w) if isinstance(w, torch.cuda.Event) else w.wait()
                    inflight[b] = None
    elif mode not in ("u4-dense", "u8"):
        local = torch.zeros((B, bins), dtype=torch.int32, device=dev)
        locals_ = [local]

        def step(i, record=False):
            count_into(local, record)
            if mode == "u32":
                done = gather(full, local, record)
                if done is not None:     # the next count rewrites `local`
                    stream.wait_event(done)

        def drain():
            pass
    else:
        # One all-gather per step of a packed slot per rank, u4-dense or u8:
        #   [B * bins counts, saturated][esc_n u32, 12 B pad][cap escapes]
        # Step i counts straight into this rank's rows of the full matrix fulls[i % 2], encodes
        # them, and all-gathers the slots (RCCL stream); step i's other ranks' rows are widened
        # into fulls[i % 2] on a side stream while step i+1 counts.  Double-buffered and ordered
        # by events (step i+2 waits for step i's widening), so every step's matrix is complete
        # and exact.
        from kmerml.kmers.matrix import slot_layout, slot_layout_u4
        if mode == "u4-dense":
            cap, P = slot_layout_u4(B, bins)
            payload = B * bins // 2
        else:
            cap, P = slot_layout(B, bins)
            payload = B * bins
        fulls = [torch.zeros((world * B, bins), dtype=torch.int32, device=dev) for _ in range(2)]
        locals_ = [f[rank * B:(rank + 1) * B] for f in fulls]
        send = [torch.zeros(P, dtype=torch.uint8, device=dev) for _ in range(2)]
        recv = [torch.empty(world * P, dtype=torch.uint8, device=dev) for _ in range(2)]
        esc_max = torch.zeros(world, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(dev)
        dec_done = [None, None]
        pending = []

        def finish(j, work):
            """Widen step j's gathered slots of the other ranks into fulls[j % 2] (side stream)."""
            if work is None:
                side.wait_stream(stream)
            with torch.cuda.stream(side):
                if work is not None:
                    side.wait_event(work)
                r = recv[j % 2]
                base = r.data_ptr()
                dst = fulls[j % 2]
                for q in range(world):
                    if q == rank:
                        continue
                    slot = base + q * P
                    if mode == "u4-dense":
                        ctx.rows_decode_u4(slot, B, bins, slot + payload + 16, cap, slot + payload,
                                           dst[q * B:].data_ptr(), side.cuda_stream)
                    else:
                        ctx.rows_decode_u8(slot, B, bins, slot + payload + 16, cap, slot + payload,
                                           1, B, dst[q * B:].data_ptr(), side.cuda_stream)
                n = r.view(world, P)[:, payload:payload + 4].contiguous().view(torch.int32)[:, 0].to(torch.int64) & 0xFFFFFFFF
                torch.maximum(esc_max, n, out=esc_max)
                ev = torch.cuda.Event()
                ev.record(side)
                dec_done[j % 2] = ev

        def step(i, record=False):
            b = i % 2
            if dec_done[b] is not None:      # step i-2's gather (send[b] -> recv[b]) and widening
                stream.wait_event(dec_done[b])
            count_into(locals_[b], record)
            sb = send[b]
            if mode == "u4-dense":
                ctx.rows_encode_u4(locals_[b].data_ptr(), B, bins, sb.data_ptr(), sb[payload + 16:].data_ptr(),
                                   cap, sb[payload:].data_ptr(), s)
            else:
                ctx.rows_encode_u8(locals_[b].data_ptr(), B, bins, sb.data_ptr(), sb[payload + 16:].data_ptr(),
                                   cap, sb[payload:].data_ptr(), s)
            work = gather(recv[b], sb, record)
            if pending:
                finish(*pending.pop())
            pending.append((i, work))

        def drain():
            while pending:
                finish(*pending.pop())

    tw = time.perf_counter()
    for i in range(a.warmup):
        step(i)
    drain()
    torch.cuda.synchronize()
    warm_run = a.warmup
    if a.min_warmup_ms > 0:
        # steps to add so that the warm-up lasts min_warmup_ms, agreed on by every rank (each step
        # holds a collective at N > 1)
        done_ms = (time.perf_counter() - tw) * 1e3
        if a.warmup == 0:
            t1 = time.perf_counter()
            step(0)
            drain()
            torch.cuda.synchronize()
            warm_run, per = 1, (time.perf_counter() - t1) * 1e3
            done_ms += per
        else:
            per = done_ms / a.warmup
        extra = min(10_000, max(0, int(np.ceil((a.min_warmup_ms - done_ms) / max(per, 1e-3)))))
        if world > 1:
            t = torch.tensor([extra], dtype=torch.int64, device=dev if not gloo else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            extra = int(t.item())
        for i in range(warm_run, warm_run + extra):
            step(i)
        drain()
        torch.cuda.synchronize()
        warm_run += extra
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if a.kernel_events == "roofline":   # an event pair costs a few us of stream time per launch
        os.environ["KMH_TIMING_ONLY"] = "k_partition,k_bucket_count,k_direct"
    ctx.timing(not a.no_kernel_events)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i, record=True)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernels = ctx.timing_report()
    ctx.timing(False)
    count_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in t_count]))
    gather_ms = None
    if t_gather:
        gather_ms = float(np.mean([x if isinstance(x, float) else x[0].elapsed_time(x[1]) for x in t_gather]))
    if world > 1:
        t = torch.tensor([elapsed, count_ms, gather_ms or 0.0], dtype=torch.float64,
                         device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, count_ms = float(t[0]), float(t[1])
        gather_ms = float(t[2]) if gather_ms is not None else None

    # sanity: every row sums to the number of valid windows (all-ACGT genomes)
    if mode == "u4" and g_local and not a.separate_encode:
        count_into(local, False)   # the fused u4-only count keeps no rows: this rank's own, untimed
        torch.cuda.synchronize()
    last = locals_[(a.steps - 1) % len(locals_)]
    if mode in ("u4-dense", "u8"):
        full = fulls[(a.steps - 1) % 2]
    if mode == "u4":   # widen the last step's compact matrix (outside the timed region) to check it
        rb = recv[(a.steps - 1) % 2]
        esc = rb.view(span, P)[:, payload:payload + 4].contiguous().view(torch.int32)[:, 0].to(torch.int64) & 0xFFFFFFFF
        esc_max = esc
        am = AssembledMatrix(G if not sim else span * B, bins, span, B, recv=rb, cap=cap, P=P)
        full = torch.zeros((span * B, bins), dtype=torch.int32, device=dev)
        for q in range(span):
            qlo, qhi = (am.G * q) // span, (am.G * (q + 1)) // span
            full[q * B:q * B + (qhi - qlo)] = am.rows(qlo, qhi)
    if sim:
        # (--sim-copy none writes only the rank's own slot: the others stay unwritten)
        nq = span if a.sim_copy == "torch" else 1
        rows = full.view(span, B, bins)[:nq, :g_local].reshape(-1, bins)
        ok_sim = all(torch.equal(full[q * B:q * B + g_local], last[:g_local]) for q in range(nq))
    elif assemble:   # every rank's block of the assembled matrix (blocks padded to B rows)
        idx = [q * B + i for q in range(world) for i in range((G * (q + 1)) // world - (G * q) // world)]
        rows = full[torch.tensor(idx, dtype=torch.long, device=full.device)]
    else:
        rows = last[:g_local]
    ok = bool(torch.all(rows.sum(1, dtype=torch.int64) == max(L - k + 1, 0)).item())
    if mode == "u32":   # this rank's block of the assembled matrix is bit-identical to its own count
        ok = ok and bool(torch.equal(full[rank * B:rank * B + g_local], last[:g_local]))
    if sim:
        ok = ok and ok_sim
    if mode in ("u4", "u4-dense", "u8") and int(esc_max.max().item()) > cap:
        raise SystemExit(f"escape list overflow ({int(esc_max.max().item())} > {cap}): use --assemble u32")
    assembly_checked = None
    if a.check_dir is not None and assemble and not sim:
        assembly_checked = check_assembly(full, last[:g_local], B, G, world, rank, k, a.check_dir)
        ok = ok and assembly_checked
    if world > 1:
        okt = torch.tensor([int(ok)], dtype=torch.int32, device=dev if not gloo else "cpu")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    c5_multi = None
    c5_full = a.config5_genome_len == 250_000_000 and a.config5_genomes_per_rank == 16
    if (world > 1 and not sim and not a.no_config5
            and ((G == 64 and L == 100_000_000 and k == 12 and not a.single_device) or not c5_full)):
        # BASELINE config 5 at this N in the same run: every rank counts its 16
        # genomes, then the matrix leg's all-to-all in the compact wire; rank 0 attaches the object
        torch.cuda.empty_cache()
        sa = argparse.Namespace(k=21, genomes=a.config5_genomes_per_rank * world, genome_len=a.config5_genome_len,
                                steps=3, warmup=1, cpu_sample=0, forward=False, backend=a.backend,
                                pmc_summary=a.pmc_summary, cpu=None, no_matrix=a.no_matrix,
                                single_device=a.single_device, matrix_wire=a.matrix_wire)
        c5_multi = run_sparse(sa, world, rank, dev, dev_index, emit=False)

    if rank == 0:
        ms = elapsed / a.steps * 1e3
        total_bases = G * L if ((assemble or world == 1) and not sim) else g_local * L * world
        value = total_bases / (elapsed / a.steps)
        # per GPU: its genomes read once + the count rows it must end up holding written once
        # compact assembly: the rank writes its own rows once; the others stay in u4 form
        algo_step = g_local * L + (G if assemble and mode != "u4" else g_local) * bins * 4
        dom = max(kernels.items(), key=lambda kv: kv[1][1]) if kernels else None
        roof = None
        if dom:
            name, (launches, tot) = dom
            per_launch_ms = tot / launches
            per_step = launches / a.steps                    # launches of this kernel per step
            if name.startswith("k_partition"):
                algo = g_local * L / per_step                # bases read once (1 B each)
            elif name == "k_bucket_count":
                algo = g_local * bins * 4 / per_step         # count rows written once
            elif name == "k_encode_u8":
                algo = B * bins * 5                          # u32 rows read, u8 rows written
            elif name == "k_decode_u8":
                algo = B * bins * 5                          # u8 rows read, u32 rows written
            elif name == "k_encode_u4":
                algo = B * bins * 4.5                        # u32 rows read, u4 rows written
            elif name == "k_decode_u4":
                algo = B * bins * 4.5                        # u4 rows read, u32 rows written
            else:
                algo = g_local * (L + bins * 4) / max(1, launches / a.steps)
            achieved = algo / (per_launch_ms * 1e-3) / 1e9
            traffic, tnote = load_traffic(a.pmc_summary, f"{name}:k{k}:L{L}:G{g_local}")
            roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                    "traffic_source": tnote,
                    "algorithmic_bytes_per_launch": algo, "mean_launch_ms": round(per_launch_ms, 4),
                    "launches_per_step": launches / a.steps}
        count_rate = g_local * L / (count_ms * 1e-3)
        out = {
            "metric": METRIC, "value": value, "unit": "bases/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "warmup_steps_run": warm_run, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": workload_name(G, L, k, world, a.single_device, a.backend),
                       "genomes": G, "genome_len": L, "k": k,
                       "parallelism": f"genome-sharded x{world}" + (f" + {mode} allgather" if assemble else ""),
                       "assembly": mode},
            "single_device": bool(a.single_device),
            "assembled_form": ({"u4": "u4 + exact escapes on every rank (rows widened on access)",
                                "u4-dense": "u32 rows on every rank (widened each step)",
                                "u8": "u32 rows on every rank (widened each step)",
                                "u32": "u32 rows on every rank"}.get(mode) if assemble else None),
            "roofline": roof,
            "step_roofline": {"algorithmic_bytes": algo_step, "achieved_GBs": round(algo_step / (ms * 1e-3) / 1e9, 1),
                              "frac": round(algo_step / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              # bases read once vs the HBM-read peak, per GPU
                              "reads_only_frac": round(g_local * L / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "count_ms_per_step_rank_max": round(count_ms, 4),
            "allgather": allgather_report(mode, world, B, bins, gather_ms, gloo, locals()),
            "count_only_bases_per_s_per_gpu": count_rate,
            "kernels": {n: {"launches": l, "total_ms": round(t, 4), "mean_ms": round(t / l, 4)}
                        for n, (l, t) in kernels.items()},
            "rows_checked": ok,
            "assembly_checked": assembly_checked,
            "cpu_baseline": cpu,
            "cpu_procs_baseline": cpu_p,
            "cpu_threads_baseline": cpu_mt,
        }
        if c5_multi is not None:
            out["config5"] = c5_multi
        if world == 1 and not sim and not a.no_config5 and G == 64 and L == 100_000_000 and k == 12:
            # BASELINE config 5 measured in the same run (its own line: bench.py --workload sparse)
            torch.cuda.empty_cache()
            sa = argparse.Namespace(k=21, genomes=a.config5_genomes_per_rank, genome_len=a.config5_genome_len,
                                    steps=3, warmup=1, cpu_sample=0, forward=False, backend=a.backend,
                                    pmc_summary=a.pmc_summary, cpu=cpu5, no_matrix=a.no_matrix, single_device=False)
            try:
                out["config5"] = run_sparse(sa, 1, 0, dev, dev_index, emit=False)
            except Exception as e:   # never lose the config-3 line over the extra measurement
                out["config5"] = {"error": f"{type(e).__name__}: {e}"}
        if world == 1 and not sim and not a.no_e2e and G == 64 and L == 100_000_000 and k == 12:
            torch.cuda.empty_cache()
            try:
                out["e2e"] = run_e2e(dev, dev_index, {12: cpu, 21: cpu5})
            except Exception as e:
                out["e2e"] = {"error": f"{type(e).__name__}: {e}"}
        if sim:
            out["config"]["workload"] = (f"projection: ONE rank of config 4 at N = {sim} on one GPU (its {g_local} of "
                                         f"{G} synthetic {L / 1e6:g} Mbp genomes, k={k}, u4 encode, the all-gather "
                                         f"modelled as {sim - 1} device copies of its slot into the others (the all-gather is in place: "
                                         f"the count writes the rank's own slot); no xGMI traffic, no other ranks)")
            out["simulated_ranks"] = sim
            out["simulated_copies"] = a.sim_copy
            out["projected_value_at_n"] = G * L / (elapsed / a.steps)
            # what the projection assumes of the wire: each rank receives the other N - 1 slots
            # once per step, hidden behind its next count, i.e. at least this rate per GPU
            # sustained over xGMI (against 7 links x XGMI_LINK_GBS)
            recv_b = (sim - 1) * P
            out["projected_xgmi"] = {"received_bytes_per_rank_per_step": recv_b,
                                     "required_GBs_per_gpu": round(recv_b / (ms * 1e-3) / 1e9, 1),
                                     "count_phase_ms": round(count_ms, 4),
                                     "required_GBs_over_count_phase": round(recv_b / (count_ms * 1e-3) / 1e9, 1),
                                     "frac_of_7_links": round(recv_b / (ms * 1e-3) / 1e9 / (7 * XGMI_LINK_GBS), 4)}
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("row-sum check failed")


YEAST_LENGTHS = [230218, 813184, 316620, 1531933, 576874, 270161, 1090940, 562643, 439888, 745751, 666816,
                 1078177, 924431, 784333, 1091291, 948066, 85779]   # config 1's 17 records


def _write_synth_fasta(ctx, dev, path, lengths, prefix):
    """A FASTA of synthetic genome 0 (generated on the device) cut into records of
    `lengths` bases, 80-column lines."""
    L = sum(lengths)
    d = torch.empty(L, dtype=torch.uint8, device=dev)
    ctx.synth_dev(d.data_ptr(), L, L, 1, SEED_BASE, torch.cuda.current_stream(dev).cuda_stream)
    seq = d.cpu().numpy()
    with open(path, "wb") as f:
        pos = 0
        for i, n in enumerate(lengths):
            body = seq[pos:pos + n]
            pos += n
            f.write(f">{prefix}{i + 1:02d}\n".encode())
            full = n // 80
            lines = np.empty((full, 81), np.uint8)
            lines[:, :80] = body[:full * 80].reshape(full, 80)
            lines[:, 80] = ord("\n")
            f.write(lines.tobytes())
            if n % 80:
                f.write(body[full * 80:].tobytes() + b"\n")


def run_e2e(dev, dev_index, cpu):
    """The drop-in end to end: the reference CLI's call pattern
    (scripts/extract_kmers.py:55-61: KmerExtractor(output_dir, compress=False) then
    extract_kmers_from_fasta(path, k_values) per genome) on synthetic FASTA files, with the
    drop-in's stage clocks (kmerml.kmers.generate.PROFILE: parse, pack, h2d, count = kernels +
    first-occurrence order + D2H, format, write, trim).  Beside it the reference's loop and
    writer (cpu_baseline: count seconds per base and save seconds per line measured on its
    sample) projected onto the same files.  Each case runs once untimed, then timed."""
    import contextlib
    import io
    import tempfile
    from kmerml.kmers import generate as kgen
    ctx = _native.context(dev_index)
    # (the last case: the class default compress=True, generate.py:10,79-91 -- gzip files)
    cases = [("yeast_standin_12.16Mbp", YEAST_LENGTHS, [8, 9, 10, 11, 12], False),
             ("yeast_standin_12.16Mbp", YEAST_LENGTHS, [21], False),
             ("yeast_standin_12.16Mbp", YEAST_LENGTHS, [8, 9, 10, 11, 12], True),
             ("synthetic_100Mbp", [100_000_000], [8, 9, 10, 11, 12], False)]
    out = {"call": "KmerExtractor(output_dir, compress=False).extract_kmers_from_fasta(fasta, k_values) "
                   "(scripts/extract_kmers.py:55-61 defaults: -k 8,9,10,11,12, no --compress); the case with "
                   "compress=True is the class default (generate.py:10), gzip-compressed k{k}.txt.gz files",
           "cases": []}
    with tempfile.TemporaryDirectory() as tmp:
        for name, lengths, ks, gz in cases:
            fa = os.path.join(tmp, f"{name}.fa")
            if not os.path.exists(fa):
                _write_synth_fasta(ctx, dev, fa, lengths, "SYN_chr" if len(lengths) > 1 else "SYN_")
            L = sum(lengths)
            ex = kgen.KmerExtractor(output_dir=os.path.join(tmp, "out"), compress=gz)
            for timed in (False, True):
                kgen.PROFILE = {}
                t0 = time.perf_counter()
                with contextlib.redirect_stdout(io.StringIO()):
                    ex.extract_kmers_from_fasta(fa, ks, organism_id=name)
                dt = time.perf_counter() - t0
            stages = {k: round(v, 4) for k, v in kgen.PROFILE.items()}
            kgen.PROFILE = None
            odir = os.path.join(tmp, "out", name)
            ext = ".txt.gz" if gz else ".txt"
            if gz:
                import gzip
                lines = sum(sum(1 for _ in gzip.open(os.path.join(odir, f"k{k}{ext}"), "rb")) for k in ks)
            else:
                lines = sum(sum(1 for _ in open(os.path.join(odir, f"k{k}{ext}"), "rb")) for k in ks)
            nbytes = sum(os.path.getsize(os.path.join(odir, f"k{k}{ext}")) for k in ks)
            case = {"input": f"{name}: {len(lengths)} record(s), {L} bases, 80-column FASTA", "k_values": ks,
                    "compress": gz,
                    "seconds": round(dt, 4), "bases_per_s": L / dt, "bases_x_k_per_s": L * len(ks) / dt,
                    "stages_s": stages, "lines_written": lines, "bytes_written": nbytes}
            ref = (cpu or {}).get(21 if ks == [21] else 12)
            if ref and not gz:   # the reference's loop + writer at the rates measured on its sample
                est = len(ks) * L / ref["value"] + lines * ref["save_seconds"] / ref["save_lines"]
                case["reference_projection"] = {
                    "seconds": round(est, 1), "bases_per_s": L / est,
                    "basis": f"cpu_baseline k={ref['k']}: count {ref['value']:.3g} bases/s per k, save "
                             f"{ref['save_seconds'] / ref['save_lines'] * 1e6:.2f} us per line (one core)",
                    "speedup": round(est / dt, 1)}
            out["cases"].append(case)
            for k in ks:
                os.remove(os.path.join(odir, f"k{k}{ext}"))
            if name.startswith("synthetic"):
                os.remove(fa)
    return out


def run_sparse(a, world, rank, dev, dev_index, emit=True):
    """Config 5: k = 21 canonical k-mers of 250 Mbp genomes counted with the device hash-table
    path (kmh_count_sparse_dev); each rank counts its contiguous block of genomes (the count step,
    no collective: the full 4^21-column matrix would not fit), then the matrix leg
    (matrix_leg): rows in code order, at N > 1 one all-to-all of code-range slices in the compact
    wire, each rank's column shard.  emit=False: return the object (rank 0) and leave the process
    group up (the dense line's config5 object)."""
    k, G, L = a.k, a.genomes, a.genome_len
    lo, hi = (G * rank) // world, (G * (rank + 1)) // world
    g_local = hi - lo
    cpu = getattr(a, "cpu", None)
    if cpu is None and rank == 0 and world == 1 and a.cpu_sample > 0:
        cpu = cpu_baseline(min(a.cpu_sample, CONFIG5_CPU_SAMPLE), k, strand="forward" if not a.forward else None)
    ctx = _native.context(dev_index)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    stride = (L + 15) // 16 * 16
    d_seq = torch.empty(max(g_local, 1) * stride, dtype=torch.uint8, device=dev)
    if stride != L:
        d_seq.fill_(ord("N"))
    if g_local:
        ctx.synth_dev(d_seq.data_ptr(), L, stride, g_local, SEED_BASE + lo, s)
    offsets = np.arange(g_local + 1, dtype=np.uint64) * np.uint64(stride)
    out_off = _native.sparse_out_offsets(offsets, k)
    cap = max(int(out_off[-1]), 1)
    d_codes = torch.empty(cap, dtype=torch.int64, device=dev)
    d_counts = torch.empty(cap, dtype=torch.int32, device=dev)
    d_nk = torch.zeros(max(g_local, 1), dtype=torch.int64, device=dev)
    canonical = 0 if a.forward else 1

    def step():
        if g_local:
            ctx.count_sparse_dev(d_seq.data_ptr(), offsets, k, canonical, d_codes.data_ptr(),
                                 d_counts.data_ptr(), d_nk.data_ptr(), s)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    os.environ["KMH_TIMING_ONLY"] = "k_sp_partition,k_sp_split,k_sp_count"
    ctx.timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernels = ctx.timing_report()
    ctx.timing(False)

    # checks: every genome's counts sum to its windows; distinct within capacity
    nk = d_nk.cpu().numpy()[:g_local]
    ok = True
    for g in range(g_local):
        a0, n = int(out_off[g]), int(nk[g])
        tot = int(d_counts[a0:a0 + n].to(torch.int64).sum().item())
        ok = ok and tot == L - k + 1 and 0 < n <= L - k + 1
    distinct = int(nk.sum())
    if world > 1:
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64,
                         device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, ok = float(t[0]), float(t[1]) == 0.0
    if rank == 0:
        ms = elapsed / a.steps * 1e3
        value = G * L / (elapsed / a.steps)
        algo_step = g_local * L + distinct * 12        # L x 1 B + distinct x 12 B
        roof = None
        if kernels:
            name, (launches, tot) = max(kernels.items(), key=lambda kv: kv[1][1])
            per_launch_ms = tot / launches
            per_step = launches / a.steps
            if name == "k_sp_partition":
                algo = g_local * L / per_step               # bases read once per launch
            elif name == "k_sp_count":
                algo = distinct * 12 / per_step             # distinct (code u64, count u32) written once
            else:
                algo = algo_step / per_step
            achieved = algo / (per_launch_ms * 1e-3) / 1e9
            traffic, tnote = load_traffic(a.pmc_summary, f"{name}:k{k}:L{L}:G{g_local}")
            roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic.get("hbm_bytes_per_launch") if traffic else None,
                    "traffic_source": tnote,
                    "algorithmic_bytes_per_launch": algo, "mean_launch_ms": round(per_launch_ms, 4),
                    "launches_per_step": per_step}
        out = {
            "metric": METRIC, "value": value, "unit": "bases/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": (("config5" if L == 250_000_000 and G == 16 * world and not
                                     getattr(a, "single_device", False) else
                                     f"rehearsal ({world} rank(s){' sharing cuda:0' if getattr(a, 'single_device', False) else ''}, "
                                     "not a config-5 measurement)")
                                    + f": {G} synthetic {L / 1e6:g} Mbp genomes, k={k} "
                                    f"{'forward' if a.forward else 'canonical'} sparse counts "
                                    f"({g_local} per GPU, hash-table path)"),
                       "genomes": G, "genome_len": L, "k": k, "parallelism": f"genome-sharded x{world}"},
            "roofline": roof,
            "step_roofline": {"algorithmic_bytes": algo_step,
                              "achieved_GBs": round(algo_step / (ms * 1e-3) / 1e9, 1),
                              "frac": round(algo_step / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "reads_only_frac": round(g_local * L / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            "distinct_kmers_rank0": distinct,
            "kernels": {n: {"launches": l, "total_ms": round(t, 4), "mean_ms": round(t / l, 4)}
                        for n, (l, t) in kernels.items()},
            "rows_checked": ok,
            "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
    mx = None
    if not getattr(a, "no_matrix", False):
        # the column-sharded matrix of these genomes, device-resident: sorted
        # rows (kmh_count_sparse_sorted_dev, back to back), at N > 1 the all-to-all of code
        # ranges in the compact wire, the shard's union and CSR indices; timed apart
        del d_codes, d_counts
        torch.cuda.empty_cache()
        mx = matrix_leg(a, world, rank, d_seq, offsets, G, k, canonical, dev)
        if rank == 0:
            out["matrix"] = mx
    if not emit:   # (the dense line's config5 object: the process group stays up for the caller)
        if not ok or (mx is not None and not mx["shard_checked"]):
            raise SystemExit("config-5 check failed (sparse counts or the sharded matrix)")
        return out if rank == 0 else None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not ok or (mx is not None and not mx["shard_checked"]):
        raise SystemExit("sparse count check failed")


def matrix_leg(a, world, rank, d_seq, offsets, G, k, canonical, dev, steps=2):
    """Time the device-resident column-sharded matrix of this rank's genomes (count in code order +
    shard: at N > 1 the code ranges' all-to-all in the compact wire format) over `steps` runs after
    one warm-up; check it globally (kmerml.kmers.matrix.shard_check: within every rank columns
    ascending and all used; across ranks the values sum to every window of every genome, so a slice
    lost or duplicated by the exchange fails, and the ranks' column ranges are in order)."""
    from kmerml.kmers import matrix as kmatrix
    t_rows, t_all, phases, shard_ph, exch = [], [], [], [], []
    m = None
    # the first run is a warm-up: its torch.empty calls reach hipMalloc (~23 GB/s for these
    # 32-48 GB buffers: 4.2 s of the first run); later runs reuse the caching allocator's blocks
    for i in range(steps + 1):
        m = None
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        ph, sph = {}, {}
        st0 = _native.context(dev.index).stats()
        codes, counts, roff = kmatrix.sorted_rows_from_device(d_seq, offsets, k, canonical, timings=ph)
        st1 = _native.context(dev.index).stats()
        ph["fallback_passes"] = st1["fallback_passes"] - st0["fallback_passes"]
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        held = [codes, counts]   # (shard_from_rows frees the rows once they are sent)
        del codes, counts
        m = kmatrix.shard_from_rows(held[0], held[1], roff, G, k, timings=sph, wire=getattr(a, "matrix_wire", "auto"),
                                    owned=held)
        del held
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t2 = time.perf_counter()
        if i:
            phases.append(ph)
            shard_ph.append(sph)
            t_rows.append((t1 - t0) * 1e3)
            t_all.append((t2 - t0) * 1e3)
            exch.append(kmatrix.LAST_EXCHANGE)
    windows = G * max(a.genome_len - k + 1, 0)
    ok, summ = kmatrix.shard_check(m, windows)
    ms = float(np.mean(t_all))
    ex_ms = float(np.mean([p.get("exchange_ms", 0.0) for p in shard_ph])) if shard_ph else 0.0
    if world > 1:
        t = torch.tensor([ms, ex_ms, 0.0 if ok else 1.0], dtype=torch.float64,
                         device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, ex_ms, ok = float(t[0]), float(t[1]), float(t[2]) == 0.0
    g_local = len(offsets) - 1
    out = {"matrix_ms": round(ms, 2), "sorted_rows_ms": round(float(np.mean(t_rows)), 2),
           "shard_ms": round(ms - float(np.mean(t_rows)), 2), "steps": steps,
           "sorted_rows_phases": {key: round(float(np.mean([p.get(key, 0.0) for p in phases])), 2)
                                  for key in phases[-1]} if phases else {},
           "shard_phases_rank0": {key: round(float(np.mean([p.get(key, 0.0) for p in shard_ph])), 2)
                                  for key in shard_ph[-1]} if shard_ph else {},
           "what": f"this rank's {g_local} genomes -> its column shard of the organisms x k-mers matrix "
                   "(features.py:96-111): kmh_count_sparse_sorted_dev (rows in code order, back to back), "
                   + ("code ranges from the rows' device cuts, one all-to-all of the slices in the compact wire "
                      "(kmh_wire_encode/decode_dev), " if world > 1 else "")
                   + "kmh_shard_union_u32_dev (columns + u32 CSR indices)",
           "ncols_rank0": int(m.columns.numel()), "nnz_rank0": m.nnz, "index_dtype": str(m.indices.dtype),
           "global": summ, "global_windows": windows, "shard_checked": ok}
    if world > 1 and exch and exch[-1]:
        e = exch[-1]
        rb = e["received_bytes"]
        gbs = rb / (ex_ms * 1e-3) / 1e9 if ex_ms > 0 else None
        out["exchange"] = dict(e, **{
            "exchange_ms_rank_max": round(ex_ms, 2),
            "received_GBs_per_gpu": round(gbs, 1) if gbs else None,
            "frac_of_7_links": round(gbs / (7 * XGMI_LINK_GBS), 4) if gbs else None,
            "bytes_per_entry": round(e["sent_bytes"] / max(1, e["raw_sent_bytes"] / 12), 3),
            "timing": ("gloo host-staged (validation only)" if a.backend == "gloo" else
                       "wall clock around one all_to_all_single (RCCL over xGMI), synchronised, max over ranks")})
    return out


def run_sparse_sim(a, dev, dev_index):
    """--workload sparse --simulate-ranks N: what ONE rank of config 5 at N GPUs does per matrix step,
    on one GPU: its 16 genomes counted in code order, cut at the N code ranges
    (bounds from the histogram of all N x 16 genomes), the slices for the other N - 1 ranks packed in
    the compact wire, the bytes that would arrive from the other ranks unpacked -- really the other
    ranks' genomes (counted, cut to this rank's range and packed before timing) -- and the union of
    this rank's shard at its N = 8 shape: R = N x 16 organism rows over 1/N of the code space.  The
    xGMI transfer itself is not run: its HBM side is modelled by a device copy of the packed bytes,
    and the line prints the bytes and the step time at a stated link rate (a projection)."""
    from kmerml.kmers import matrix as kmatrix
    N, k, L = a.simulate_ranks, a.k, a.genome_len
    gpr = a.genomes          # genomes per rank (--genomes; 16 by default, config 5's 128 / 8)
    G = N * gpr
    canonical = 0 if a.forward else 1
    ctx = _native.context(dev_index)
    s = torch.cuda.current_stream(dev).cuda_stream
    stride = (L + 15) // 16 * 16
    d_seq = torch.empty(gpr * stride, dtype=torch.uint8, device=dev)
    if stride != L:
        d_seq.fill_(ord("N"))
    offsets = np.arange(gpr + 1, dtype=np.uint64) * np.uint64(stride)

    def batch_rows(b):
        ctx.synth_dev(d_seq.data_ptr(), L, stride, gpr, SEED_BASE + b * gpr, s)
        return kmatrix.sorted_rows_from_device(d_seq, offsets, k, canonical)

    t_setup = time.perf_counter()
    hist = None
    for b in range(N):   # the global histogram the all-reduce would give
        codes, counts, roff = batch_rows(b)
        h = kmatrix._row_histogram(codes, roff, k)
        hist = h if hist is None else hist + h
        del codes, counts
    bounds = kmatrix._splitters_from_hist(hist.cpu().numpy(), k, N)
    # what arrives from the other ranks: their genomes' slices of range 0, packed by them
    parts, rs_n, rs_b = [], [], []
    for b in range(1, N):
        codes, counts, roff = batch_rows(b)
        send_len, starts = kmatrix.shard_plan(codes, roff, bounds, b)
        st, sn = starts[:, 0].astype(np.uint64), send_len[:, 0].astype(np.uint64)
        sb = ctx.wire_size_dev(codes.data_ptr(), counts.data_ptr(), st, sn, s)
        buf = torch.empty(max(int(sb.sum()), 16), dtype=torch.uint8, device=dev)
        ctx.wire_encode_dev(codes.data_ptr(), counts.data_ptr(), st, sn, buf.data_ptr(), int(sb.sum()), s)
        parts.append(buf[:int(sb.sum())])
        rs_n += sn.tolist()
        rs_b += sb.tolist()
        del codes, counts
    recv = torch.cat(parts)
    del parts
    ctx.synth_dev(d_seq.data_ptr(), L, stride, gpr, SEED_BASE, s)   # this rank's genomes, resident
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    def step(ph):
        t = [time.perf_counter()]

        def mark(name):
            torch.cuda.synchronize()
            now = time.perf_counter()
            ph[name] = ph.get(name, 0.0) + (now - t[0]) * 1e3
            t[0] = now
        codes, counts, roff = kmatrix.sorted_rows_from_device(d_seq, offsets, k, canonical)
        mark("sorted_rows_ms")
        h = kmatrix._row_histogram(codes, roff, k)   # (its all-reduce is not modelled)
        send_len, starts = kmatrix.shard_plan(codes, roff, bounds, 0)
        del h
        mark("plan_ms")
        st = np.concatenate([starts[:, q] for q in range(1, N)]).astype(np.uint64)
        sn = np.concatenate([send_len[:, q] for q in range(1, N)]).astype(np.uint64)
        sb = ctx.wire_size_dev(codes.data_ptr(), counts.data_ptr(), st, sn, s)
        nbytes = int(sb.sum())
        send = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
        ctx.wire_encode_dev(codes.data_ptr(), counts.data_ptr(), st, sn, send.data_ptr(), nbytes, s)
        mark("encode_ms")
        # receive layout: genome-major, this rank's genomes first (it is rank 0)
        gl = np.concatenate([send_len[:, 0], np.array(rs_n, np.int64)])
        indptr = np.zeros(G + 1, np.int64)
        np.cumsum(gl, out=indptr[1:])
        total = int(indptr[-1])
        rc = torch.empty(total, dtype=torch.int64, device=dev)
        rn = torch.empty(total, dtype=torch.int32, device=dev)
        for j in range(gpr):
            a0, m_, d = int(starts[j, 0]), int(send_len[j, 0]), int(indptr[j])
            rc[d:d + m_].copy_(codes[a0:a0 + m_])
            rn[d:d + m_].copy_(counts[a0:a0 + m_])
        del codes, counts
        mark("own_copy_ms")
        if a.sim_copy == "torch":   # the wire's HBM side: the packed bytes written once more on arrival
            scratch = torch.empty_like(recv)
            scratch.copy_(recv)
            del scratch
        del send
        mark("wire_model_ms")
        ctx.wire_decode_dev(recv.data_ptr(), recv.numel(), np.array(rs_n, np.uint64), np.array(rs_b, np.uint64),
                            indptr[gpr:G].astype(np.uint64), rc.data_ptr(), rn.data_ptr(), s)
        mark("decode_ms")
        columns = torch.empty(total, dtype=torch.int64, device=dev)
        indices = torch.empty(total, dtype=torch.int32, device=dev)
        ncols = ctx.shard_union_dev(rc.data_ptr(), indptr.astype(np.uint64), bounds[0], bounds[1] - 1,
                                    columns.data_ptr(), indices.data_ptr(), s, idx32=True)
        mark("union_ms")
        m = kmatrix.ShardedSparseMatrix(k, G, bounds[0], bounds[1], columns[:ncols], indptr, indices, rn, 0, N)
        return m, nbytes, total

    times, phs = [], []
    for i in range(a.steps + 1):
        ph = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m, sent, total = step(ph)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        if i:
            times.append(dt)
            phs.append(ph)
        if i < a.steps:
            del m
    ok = m.all_columns_used() and m.columns_ascending()
    cols = m.columns
    # every entry of range 0 of all N x 16 genomes arrived: the rows' cuts of range 0 summed
    want_entries = int(hist.cpu().numpy()[:bounds[1] >> max(2 * k - 16, 0)].sum())
    ok = ok and total == want_entries
    ms = float(np.mean(times))
    received = int(recv.numel())
    rate = 0.5 * 7 * XGMI_LINK_GBS   # GB/s assumed for the projection: half of the 7 links' peak
    xfer_ms = max(sent, received) / (rate * 1e9) * 1e3
    proj_ms = ms + xfer_ms
    out = {"metric": METRIC, "value": None, "unit": "bases/s", "n_gpus": 1, "steps": a.steps, "warmup": 1,
           "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic",
           "config": {"workload": (f"projection: ONE rank of config 5's matrix at N = {N} on one GPU (its {gpr} of "
                                   f"{G} synthetic {L / 1e6:g} Mbp genomes, k={k} "
                                   f"{'forward' if a.forward else 'canonical'}: count in code order, cut, pack the "
                                   f"slices of the other {N - 1} ranks, unpack the other ranks' real slices of its "
                                   f"range, union at R = {G} rows); no xGMI traffic, no other ranks"),
                      "genomes": G, "genome_len": L, "k": k, "parallelism": f"code-range sharded x{N} (simulated)"},
           "simulated_ranks": N, "simulated_copies": a.sim_copy,
           "phases_ms": {key: round(float(np.mean([p[key] for p in phs])), 2) for key in phs[-1]},
           "shard": {"rows": G, "entries": total, "columns": int(cols.numel()), "lo_code": bounds[0],
                     "hi_code": bounds[1], "checked": ok},
           "exchange": {"wire": "compact", "sent_bytes": sent, "received_bytes": received,
                        "raw_received_bytes": int(sum(rs_n)) * 12,
                        "bytes_per_entry": round(received / max(1, sum(rs_n)), 3),
                        "assumed_xgmi_GBs": rate, "transfer_ms_at_assumed_rate": round(xfer_ms, 2),
                        "required_GBs_to_hide_in_step": round(received / (ms * 1e-3) / 1e9, 1)},
           "projected_ms_per_step": round(proj_ms, 2),
           "projected_value_at_n": G * L / (proj_ms * 1e-3),
           "setup_s": round(setup_s, 1)}
    print(json.dumps(out), flush=True)
    if not ok:
        raise SystemExit("simulated shard check failed")


if __name__ == "__main__":
    from kmerml.utils.devmem import run_guarded
    run_guarded(main)
