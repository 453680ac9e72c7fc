"""Per-organism k-mer feature CSVs, vectorised -- drop-in for the reference's
kmerml/kmers/statistics.py (row f4).

The reference builds one Python dict per k-mer with ``DataFrame.iterrows`` (37 us per row,
about 10 minutes per organism for a dense k = 12 file, statistics.py:149-186).  Every
feature is a pure function of the k-mer label, so here they are computed for all labels of
a file at once with numpy over one concatenated code-point buffer.  The output files,
columns, dtypes and values are the reference's, including its quirks:

* labels are read with the same pandas calls (statistics.py:253-272), so integer type
  inference drops the leading zeros (the A's) of labels that fit int64/uint64 (k <= 19,
  and k = 20 files whose labels all fit), and a label is decoded with 0->A 1->T 2->C 3->G
  only if ``str(label).isdigit()`` (statistics.py:157, :248-251);
* Shannon entropy is summed in the iteration order of ``set(kmer)`` in this interpreter
  (statistics.py:216-224).  That order depends only on the sequence of distinct characters
  in first-appearance order, so it is evaluated once per such pattern, and log2 comes from
  ``math.log2`` on the distinct probabilities -- the sums are bit-identical to the
  reference's in the same process;
* the CpG observed/expected ratio, GC percent, presence and repeat flags follow
  statistics.py:188-238 operation for operation (same IEEE operation order).
"""
import math
import re
import time
from collections import defaultdict
from pathlib import Path

import numpy as np
import pandas as pd

from kmerml.utils.progress import progress_bar

DEFAULT_FEATURES = ['base_counts', 'gc_content', 'cpg_sites', 'entropy', 'repeats', 'presence']
_DECODE = str.maketrans({str(d): 'N' for d in range(10)} | {'0': 'A', '1': 'T', '2': 'C', '3': 'G'})


class KmerFeatureExtractor:
    """Extract machine-learning features from k-mer files (statistics.py:9-33)."""

    def __init__(self, input_paths=None, output_dir=None, metadata_file=None):
        self.input_paths = [Path(p) for p in input_paths] if input_paths else []
        self.output_dir = Path(output_dir) if output_dir else Path("kmer_features")
        self.output_dir.mkdir(exist_ok=True, parents=True)
        self.metadata = None
        if metadata_file:
            from kmerml.utils.genome_metadata import GenomeMetadataManager
            self.metadata_manager = GenomeMetadataManager(metadata_file)

    def add_paths(self, paths):
        self.input_paths.extend([Path(p) for p in paths])

    def extract_features(self, required_features=None):
        """Write <output_dir>/<organism>_kmer_features.csv per organism (statistics.py:35-72)."""
        if required_features is None:
            required_features = list(DEFAULT_FEATURES)
        files_by_organism = self._group_files_by_organism()
        total = len(files_by_organism)
        start = time.time()
        output_files = {}
        for i, (organism, files) in enumerate(files_by_organism.items(), 1):
            output_files[organism] = self._process_organism_kmers(organism, files, required_features)
            start = progress_bar(i, total, start_time=start, title="Organisms processed")
        return output_files

    def _group_files_by_organism(self):
        """Same grouping and order as statistics.py:74-93."""
        groups = defaultdict(list)
        for path in self.input_paths:
            if path.is_file():
                groups[path.parent.name].append(path)
            elif path.is_dir():
                for org_dir in path.iterdir():
                    if org_dir.is_dir():
                        for kmer_file in org_dir.glob("k*.txt*"):
                            groups[org_dir.name].append(kmer_file)
        return groups

    def _process_organism_kmers(self, organism, kmer_files, required_features):
        genome_size = None
        if hasattr(self, 'metadata_manager'):
            genome_size = self.metadata_manager.get_genome_size(organism)
        blocks = []
        total = len(kmer_files)
        start = time.time()
        for i, kmer_file in enumerate(kmer_files, 1):
            k_val = self._extract_k_from_filename(kmer_file.name)
            if k_val is None:
                print(f"Warning: Could not extract k value from {kmer_file}")
                continue
            df = self._load_kmer_file(kmer_file)
            blocks.append(self.feature_block(df, k_val, required_features))
            start = progress_bar(i, total, start_time=start, title="K values processed")
        blocks = [b for b in blocks if b.nrows]
        if not blocks:
            print(f"No features extracted for {organism}")
            return None
        if genome_size:
            for b in blocks:
                b.cols['genome_size'] = np.full(b.nrows, genome_size)
        output_file = self.output_dir / f"{organism}_kmer_features.csv"
        write_feature_csv(blocks, output_file)
        print(f"Created feature CSV for {organism}: {output_file}")
        return output_file

    # ------------------------------------------------------------------ features
    @staticmethod
    def decode_labels(column):
        """Labels as statistics.py:157 sees them: digit strings decoded, others unchanged."""
        values = column.to_numpy()
        if values.dtype.kind in 'iu':            # integer labels: every str() is all digits
            text = '\n'.join(values.astype(str).tolist()).translate(_DECODE)
            return np.array(text.split('\n') if len(values) else [], dtype=object)
        out = np.empty(len(values), dtype=object)
        for i, v in enumerate(values):
            s = str(v)
            out[i] = s.translate(_DECODE) if s.isdigit() else v
        return out

    @classmethod
    def feature_frame(cls, df, k_val, required_features):
        """The rows statistics.py:149-186 would produce for one k-mer file, as a DataFrame."""
        return cls.feature_block(df, k_val, required_features).frame()

    @classmethod
    def feature_block(cls, df, k_val, required_features):
        """feature_frame's columns without the DataFrame (a FeatureBlock): the label column stays
        as codes when every label is an integer-parsed k-mer, for the native CSV writer."""
        n = len(df)
        codes = label_codes(df['kmer'].to_numpy(), k_val) if n else None
        cols = {'kmer': None, 'count': df['count'].to_numpy(), 'k': np.full(n, k_val, dtype=np.int64)}
        block = FeatureBlock(cols, n, df['kmer'], codes, k_val)
        if n == 0:
            return block
        if codes is not None:   # every label is a k-mer: features computed per code
            f = code_features_of(k_val, codes)
        else:
            f = label_features([str(x) for x in block.labels()])
        if 'gc_content' in required_features:
            cols['gc_percent'] = f['gc_percent']
        if 'base_counts' in required_features:
            for b in 'ACGT':
                cols[f'{b}_count'] = f[f'{b}_count']
        if 'presence' in required_features:
            for b in 'ACGT':
                cols[f'{b}_present'] = (f[f'{b}_count'] > 0).astype(np.int64)
        if 'cpg_sites' in required_features:
            cols['cpg_count'] = f['cpg_count']
            cols['cpg_obs_exp'] = f['cpg_obs_exp']
        if 'entropy' in required_features:
            cols['shannon_entropy'] = f['shannon_entropy']
            cols['normalized_entropy'] = f['shannon_entropy'] / 2.0
        if 'repeats' in required_features:
            cols['has_repeat'] = f['has_repeat']
        return block

    # ------------------------------------------------------------------ helpers
    def _extract_k_from_filename(self, filename):
        match = re.search(r'k(\d+)', filename)
        return int(match.group(1)) if match else None

    def _decode_kmer(self, encoded_kmer):
        return str(encoded_kmer).translate(_DECODE)

    def _load_kmer_file(self, filepath):
        """The reference's loader, call for call (statistics.py:253-272): the header
        guess and the integer type inference of the label column are part of its output."""
        compression = 'gzip' if str(filepath).endswith('.gz') else None
        try:
            df = pd.read_csv(filepath, sep='\t', compression=compression)
            if 'kmer' not in df.columns and 'count' not in df.columns:
                df = pd.read_csv(filepath, sep='\t', header=None, names=['kmer', 'count'], compression=compression)
        except Exception:
            df = pd.read_csv(filepath, sep='\t', header=None, names=['kmer', 'count'], compression=compression)
        return df


class FeatureBlock:
    """The feature rows of one k-mer file (statistics.py:149-186): column name -> numpy array,
    in the reference's column order.  The 'kmer' column is kept as the file's label column and,
    when every label is an integer-parsed k-mer, its codes (label_codes), so the native writer
    prints the labels from the codes without building a Python string per row."""

    def __init__(self, cols, nrows, raw_labels, codes, k):
        self.cols, self.nrows, self.raw_labels, self.codes, self.k = cols, nrows, raw_labels, codes, k

    def labels(self):
        """The 'kmer' column as statistics.py:157 sees it (decode_labels)."""
        return KmerFeatureExtractor.decode_labels(self.raw_labels)

    def frame(self):
        cols = dict(self.cols)
        cols['kmer'] = self.labels() if self.nrows else np.empty(0, dtype=object)
        return pd.DataFrame(cols)


def _native_columns(block):
    """(kind, data, aux) per column for _native.csv_format, or None if a column has a dtype the
    native writer does not print the way pandas does."""
    from kmerml import _native
    out = []
    for name, v in block.cols.items():
        if name == 'kmer':
            if block.codes is not None:
                out.append((_native.CSV_LABEL, block.codes.astype(np.uint64), block.k))
                continue
            labels = block.labels()
            if not all(type(x) is str for x in labels):
                return None
            enc = [x.encode('utf-8') for x in labels]
            off = np.zeros(len(enc) + 1, dtype=np.uint64)
            np.cumsum(np.fromiter(map(len, enc), dtype=np.uint64, count=len(enc)), out=off[1:])
            out.append((_native.CSV_STR, b''.join(enc), off))
            continue
        v = np.asarray(v)
        if v.dtype.kind == 'i':
            out.append((_native.CSV_I64, v, None))
        elif v.dtype.kind == 'u':
            out.append((_native.CSV_U64, v, None))
        elif v.dtype == np.float64:
            out.append((_native.CSV_F64, v, None))
        else:
            return None
    return out


def _dtype_signature(block):
    return tuple((name, 'O' if name == 'kmer' else np.asarray(v).dtype.str) for name, v in block.cols.items())


def write_feature_csv(blocks, path):
    """``pd.concat([b.frame() for b in blocks]).to_csv(path, index=False)``, with the rows of
    each block formatted by the native writer (kmh_csv_format: Python's float repr, integer
    str(), the k-mer labels printed from their codes).  A block holding a value pandas writes
    differently (NaN, inf, text that needs quoting) is written by pandas itself; blocks whose
    column dtypes differ (pandas would then upcast the concatenated column) are all written by
    pandas."""
    from kmerml import _native
    if len({_dtype_signature(b) for b in blocks}) > 1 or any(q in name for name in blocks[0].cols for q in _NEEDS_QUOTES):
        frames = [b.frame() for b in blocks]
        (pd.concat(frames, ignore_index=True) if len(frames) > 1 else frames[0]).to_csv(path, index=False)
        return
    with open(path, 'wb') as f:
        f.write((','.join(blocks[0].cols) + '\n').encode())
        for b in blocks:
            cols = _native_columns(b)
            text = _native.csv_format(cols, b.nrows) if cols is not None else None
            if text is None:
                text = b.frame().to_csv(index=False, header=False).encode('utf-8')
            f.write(text)


_NEEDS_QUOTES = (',', '"', '\n', '\r')


def csv_text(df):
    """``df.to_csv(index=False)`` text, or None where pandas would quote or write NaN/inf.

    pandas turns float64 columns into text with numpy's shortest round-trip repr -- the same
    digits as Python's float repr -- but at ~2 us per value; repr on a list is ~20x faster.
    """
    cols = []
    for name in df.columns:
        v = df[name].to_numpy()
        if v.dtype.kind in 'iu':
            cols.append(list(map(str, v.tolist())))
        elif v.dtype.kind == 'f':
            if not np.isfinite(v).all():
                return None
            cols.append(list(map(repr, v.tolist())))
        elif v.dtype.kind == 'O' and all(type(x) is str for x in v):
            if any(q in x for x in v for q in _NEEDS_QUOTES):
                return None
            cols.append(v.tolist())
        else:
            return None
    header = [str(c) for c in df.columns]
    if any(q in h for h in header for q in _NEEDS_QUOTES):
        return None
    body = '\n'.join(map(','.join, zip(*cols)))
    return ','.join(header) + '\n' + (body + '\n' if len(df) else '')


def write_csv(df, path):
    """Write ``df`` exactly as ``df.to_csv(path, index=False)`` would."""
    text = csv_text(df)
    if text is None:
        df.to_csv(path, index=False)
        return
    with open(path, 'w', newline='') as f:
        f.write(text)


_DIGIT_CODE = np.array([0, 3, 1, 2, -1, -1, -1, -1, -1, -1], dtype=np.int64)   # file digit -> A0 C1 G2 T3


def label_codes(values, k):
    """2-bit codes (A0 C1 G2 T3, first base most significant) of integer-parsed labels of a
    k{k}.txt file, or None unless every label is one: an integer whose decimal digits are the
    reference's A0 T1 C2 G3 digits of a k-mer with its leading A's (zeros) lost
    (statistics.py:253-272 parses them so).  Code c's table row then holds the features of
    exactly the label the reference computes them on."""
    if values.dtype.kind not in 'iu' or not 1 <= k <= 19 or len(values) == 0:
        return None
    v = values.astype(np.int64)
    if v.min() < 0:
        return None
    codes = np.zeros(len(v), dtype=np.int64)
    for i in range(k):
        d = _DIGIT_CODE[v % 10]
        if (d < 0).any():
            return None
        codes |= d << (2 * i)
        v //= 10
    return codes if not v.any() else None


_TABLES = {}          # k -> the table of feature_table(k); only the last k is kept
_TABLE_MAX_K = 12     # a full table is 4^k rows (k = 12: 16.7 M rows, ~30 temporaries of 134 MB)


def code_features_of(k, codes):
    """Feature columns for the integer-label codes of one k{k}.txt file.  A dense file (k <=
    12 and at least 1/8 of the 4^k codes present) takes rows of the per-k table; any other
    file (sparse k = 13..19 files: a few distinct k-mers out of 4^k) computes the features of
    its distinct codes only, so memory follows the file, not 4^k."""
    if k <= _TABLE_MAX_K and (1 << (2 * k)) <= 8 * len(codes):
        t = feature_table(k)
        return {name: col[codes] for name, col in t.items()}
    uniq, inv = np.unique(codes, return_inverse=True)
    t = _code_features(k, uniq)
    return {name: col[inv] for name, col in t.items()}


def feature_table(k):
    """The statistics.py:188-238 features of every label of a dense k (the compat label of each
    of the 4^k codes: the k-mer with its leading A's stripped, one kept for A...A), computed
    once per k on the GPU (torch on cuda; on the CPU without one) and indexed by code (k <= 12;
    the last table is cached)."""
    if k in _TABLES:
        return _TABLES[k]
    if not 1 <= k <= _TABLE_MAX_K:
        raise ValueError(f"feature_table: 1 <= k <= {_TABLE_MAX_K} (got {k}); use code_features_of")
    table = _code_features(k, None)
    _TABLES.clear()
    _TABLES[k] = table
    return table


def _order_lut():
    """625 x 4 int32: for the first-appearance pattern key of a label (present bases A0 C1 G2 T3
    in order of first appearance, as base-5 digits b + 1, absent ones 0), the bases in the order
    this interpreter's set() iterates them (-1-padded)."""
    from itertools import permutations
    lut = np.full((625, 4), -1, dtype=np.int32)
    letters = 'ACGT'
    for m in range(1, 5):
        for pat in permutations(range(4), m):
            key = 0
            for r in range(4):
                key = key * 5 + (pat[r] + 1 if r < m else 0)
            seq = [letters.index(ch) for ch in _entropy_order(''.join(letters[b] for b in pat))]
            lut[key, :len(seq)] = seq
    return lut


def _log2_table(k):
    """(k + 1) x (k + 1) float64: math.log2(n / L) at [n][L] (the reference's log2 of each prob)."""
    lg = np.zeros((k + 1, k + 1), dtype=np.float64)
    for L in range(1, k + 1):
        for n in range(1, L + 1):
            lg[n, L] = math.log2(n / L)
    return lg


def _code_features_hip(k, codes):
    """_code_features on the HIP device: one thread per code (kmh_feature_columns_dev,
    csrc/kmh_features.hip), the same operations rounded once each."""
    import torch

    from kmerml import _native
    dev = torch.device("cuda", torch.cuda.current_device())
    n = (1 << (2 * k)) if codes is None else len(codes)
    d_codes = None if codes is None else torch.from_numpy(np.ascontiguousarray(codes, dtype=np.int64)).to(dev)
    d_order = torch.from_numpy(_order_lut()).to(dev)
    d_lg = torch.from_numpy(_log2_table(k)).to(dev)
    cnt = torch.empty((4, n), dtype=torch.int64, device=dev)
    cpg = torch.empty(n, dtype=torch.int64, device=dev)
    rep = torch.empty(n, dtype=torch.int64, device=dev)
    gc = torch.empty(n, dtype=torch.float64, device=dev)
    oe = torch.empty(n, dtype=torch.float64, device=dev)
    ent = torch.empty(n, dtype=torch.float64, device=dev)
    ctx = _native.context(dev.index)
    ctx.feature_columns_dev(d_codes.data_ptr() if d_codes is not None else None, n, k, d_order.data_ptr(),
                            d_lg.data_ptr(), cnt.data_ptr(), cpg.data_ptr(), rep.data_ptr(), gc.data_ptr(),
                            oe.data_ptr(), ent.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    cnt = cnt.cpu().numpy()
    return {'A_count': cnt[0], 'C_count': cnt[1], 'G_count': cnt[2], 'T_count': cnt[3],
            'cpg_count': cpg.cpu().numpy(), 'has_repeat': rep.cpu().numpy(), 'gc_percent': gc.cpu().numpy(),
            'cpg_obs_exp': oe.cpu().numpy(), 'shannon_entropy': ent.cpu().numpy()}


def _hip_library_loads():
    """True if libkmerhip.so loads (the feature kernel needs it); a host with a GPU but no HIP
    build keeps the torch path of this CPU-side consumer."""
    from kmerml import _native
    try:
        _native.lib()
        return True
    except (ImportError, OSError):
        return False


def _code_features(k, codes):
    """statistics.py:188-238 for the compat labels of `codes` (None: all 4^k codes).  Same
    IEEE operations as the reference, per value: gc = (g + c) / L * 100; expected =
    c / L * (g / L) * (L - 1); entropy summed in set(kmer) order (_entropy_order per
    first-appearance pattern) with math.log2 of the same quotients.  On a HIP device the
    hand-written kernel computes them (_code_features_hip); on a host without one, torch on
    the CPU (this consumer of the k-mer files is a CPU program in the reference)."""
    import torch

    if torch.cuda.is_available() and torch.version.hip and _hip_library_loads():
        return _code_features_hip(k, codes)
    dev = torch.device("cpu")
    i64 = torch.int64
    if codes is None:
        c = torch.arange(1 << (2 * k), dtype=i64, device=dev)
    else:
        c = torch.as_tensor(np.ascontiguousarray(codes, dtype=np.int64)).to(dev)
    # stripped length m: significant base-4 digits (at least 1)
    m = torch.ones_like(c)
    for j in range(1, k):
        m += (c >= (1 << (2 * j))).to(i64)
    digit = [(c >> (2 * (k - 1 - i))) & 3 for i in range(k)]
    valid = [(k - i) <= m for i in range(k)]                       # position i is in the label
    cnt = [torch.zeros_like(c) for _ in range(4)]
    first = [torch.full_like(c, 1 << 20) for _ in range(4)]
    for i in range(k):
        for b in range(4):
            hit = valid[i] & (digit[i] == b)
            cnt[b] += hit.to(i64)
            first[b] = torch.where(hit & (first[b] > i), torch.full_like(c, i), first[b])
    cpg = torch.zeros_like(c)
    rep = torch.zeros(c.shape, dtype=torch.bool, device=dev)
    for i in range(k - 1):
        cpg += (valid[i] & (digit[i] == 1) & (digit[i + 1] == 2)).to(i64)
    for i in range(k - 3):
        rep |= valid[i] & (digit[i] == digit[i + 2]) & (digit[i + 1] == digit[i + 3])
    Lf = m.to(torch.float64)
    A, C, G, T = cnt
    out = {'A_count': A, 'C_count': C, 'G_count': G, 'T_count': T, 'cpg_count': cpg,
           'has_repeat': rep.to(i64)}
    out['gc_percent'] = ((G + C).to(torch.float64) / Lf) * 100
    c_freq, g_freq = C.to(torch.float64) / Lf, G.to(torch.float64) / Lf
    prod = c_freq * g_freq
    expected = torch.where(prod > 0, prod * (Lf - 1), torch.full_like(prod, 0.001))
    out['cpg_obs_exp'] = torch.where(expected > 0, cpg.to(torch.float64) / expected, torch.zeros_like(prod))
    # entropy: first-appearance pattern -> the set order of this interpreter
    key = torch.zeros_like(c)
    order_rank = torch.stack(first).argsort(dim=0, stable=True)      # letters by first position
    present_sorted = torch.stack(first).gather(0, order_rank) < (1 << 20)
    for r in range(4):
        key = key * 5 + torch.where(present_sorted[r], order_rank[r] + 1, torch.zeros_like(c))
    lut_order = torch.from_numpy(_order_lut().astype(np.int64)).to(dev)
    lg = torch.from_numpy(_log2_table(k)).to(dev)
    cnt_t = torch.stack(cnt)
    ent = torch.zeros_like(Lf)
    for r in range(4):
        b = lut_order[key, r]
        has = b >= 0
        n = cnt_t.gather(0, b.clamp(min=0)[None])[0]
        p = n.to(torch.float64) / Lf
        term = p * lg[n, m]                       # one rounding, as prob * math.log2(prob)
        ent = torch.where(has, ent - term, ent)
    out['shannon_entropy'] = ent
    return {name: v.cpu().numpy() for name, v in out.items()}


def _entropy_order(pattern):
    """Iteration order of set(kmer) for a k-mer whose distinct characters first appear in
    the order `pattern` (CPython's set layout depends only on that insertion sequence)."""
    return list(set(pattern))


def label_features(labels):
    """Vectorised statistics.py:188-238 for a list of label strings.

    Returns int64 arrays A/C/G/T_count, cpg_count, has_repeat and float64 arrays gc_percent,
    cpg_obs_exp, shannon_entropy.
    """
    n = len(labels)
    L = np.fromiter((len(s) for s in labels), dtype=np.int64, count=n)
    cp = np.frombuffer(''.join(labels).encode('utf-32-le'), dtype=np.uint32)
    ends = np.cumsum(L)
    starts = ends - L
    nonempty = L > 0
    st = np.minimum(starts, max(len(cp) - 1, 0))

    def seg_sum(x):   # per-label sums of an indicator over the label's positions
        if len(x) == 0:
            return np.zeros(n, dtype=np.int64)
        s = np.add.reduceat(x.astype(np.int64), st)
        return np.where(nonempty, s, 0)

    out = {}
    counts = {}
    for b in 'ACGT':
        counts[b] = seg_sum(cp == ord(b))
        out[f'{b}_count'] = counts[b]
    Lf = L.astype(np.float64)
    with np.errstate(divide='ignore', invalid='ignore'):
        gc = counts['G'] + counts['C']
        out['gc_percent'] = np.where(nonempty, (gc / Lf) * 100, 0.0)
        # CpG: 'CG' at i and i+1 inside one label
        pair = np.zeros(len(cp), dtype=bool)
        if len(cp) > 1:
            pair[:-1] = (cp[:-1] == ord('C')) & (cp[1:] == ord('G'))
        pair[ends[nonempty] - 1] = False
        cpg = seg_sum(pair)
        out['cpg_count'] = cpg
        c_freq = np.where(nonempty, counts['C'] / Lf, 0.0)
        g_freq = np.where(nonempty, counts['G'] / Lf, 0.0)
        prod = c_freq * g_freq
        expected = np.where(prod > 0, prod * (Lf - 1), 0.001)
        out['cpg_obs_exp'] = np.where(expected > 0, cpg / expected, 0.0)
        # dinucleotide repeat: kmer[i:i+2] == kmer[i+2:i+4] for some i <= len - 4
        rep = np.zeros(len(cp), dtype=bool)
        if len(cp) > 3:
            rep[:-3] = (cp[:-3] == cp[2:-1]) & (cp[1:-2] == cp[3:])
        pos = np.arange(len(cp), dtype=np.int64) - np.repeat(starts, L)
        rep &= pos <= np.repeat(L, L) - 4
        out['has_repeat'] = (seg_sum(rep) > 0).astype(np.int64)
    out['shannon_entropy'] = _entropy(labels, cp, L, starts, nonempty, pos)
    return out


def _entropy(labels, cp, L, starts, nonempty, pos):
    """statistics.py:214-224 for every label, in set(kmer) order."""
    n = len(labels)
    ent = np.zeros(n, dtype=np.float64)
    alphabet = np.unique(cp)
    if len(alphabet) > 8:    # general text labels: the reference's scalar formula per label
        for i, s in enumerate(labels):
            e = 0
            for base, c in {b: s.count(b) for b in set(s)}.items():
                p = c / len(s)
                e -= p * math.log2(p) if p > 0 else 0
            ent[i] = e
        return ent
    big = np.int64(1) << 40
    st = np.minimum(starts, max(len(cp) - 1, 0))
    first = np.empty((len(alphabet), n), dtype=np.int64)
    cnt = np.empty((len(alphabet), n), dtype=np.int64)
    for j, a in enumerate(alphabet):
        hit = cp == a
        first[j] = np.where(nonempty, np.minimum.reduceat(np.where(hit, pos, big), st), big) if len(cp) else big
        cnt[j] = np.where(nonempty, np.add.reduceat(hit.astype(np.int64), st), 0) if len(cp) else 0
    # pattern = present characters in first-appearance order, as one integer key
    order = np.argsort(first, axis=0, kind='stable')
    present = np.take_along_axis(first, order, axis=0) < big
    key = np.zeros(n, dtype=np.int64)
    for r in range(len(alphabet)):
        key = key * (len(alphabet) + 1) + np.where(present[r], order[r] + 1, 0)
    Lf = L.astype(np.float64)
    for kv in np.unique(key[nonempty]):
        rows = np.nonzero((key == kv) & nonempty)[0]
        r0 = rows[0]
        pat = ''.join(chr(alphabet[order[r, r0]]) for r in range(len(alphabet)) if present[r, r0])
        e = np.zeros(len(rows), dtype=np.float64)
        for ch in _entropy_order(pat):
            j = int(np.searchsorted(alphabet, ord(ch)))
            p = cnt[j, rows] / Lf[rows]
            uniq, inv = np.unique(p, return_inverse=True)
            lg = np.array([math.log2(x) for x in uniq.tolist()], dtype=np.float64)
            e = e - p * lg[inv]
        ent[rows] = e
    return ent
