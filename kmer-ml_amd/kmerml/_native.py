"""ctypes binding to libkmerhip.so (the C ABI declared in include/kmerhip.h).

There is no CPU fallback: if the library or a HIP device is missing, every counting
call raises.  ctypes releases the GIL for the duration of each foreign call.
"""
import ctypes
import os
import threading

import numpy as np

DEFAULT_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libkmerhip.so")
# KMH_LIB_PATH: A/B profiling of another build of the same ABI (profiles/); every symbol of
# SIGNATURES must resolve, and a warning names the build id of the library loaded instead
LIB_PATH = os.environ.get("KMH_LIB_PATH") or DEFAULT_LIB_PATH

KMH_OK = 0
KMH_ERR_INVALID = -1
KMH_ERR_HIP = -2
KMH_ERR_NOMEM = -3
KMH_ERR_UNSUPPORTED = -4
KMH_ERR_IO = -5
MAX_DENSE_K = 12
MAX_SPARSE_K = 32

_c = ctypes
_vp = _c.c_void_p
_u64 = _c.c_uint64
_u64p = _c.POINTER(_c.c_uint64)

# (name, restype, argtypes) for every symbol of include/kmerhip.h
SIGNATURES = [
    ("kmh_version", _c.c_char_p, []),
    ("kmh_build_id", _c.c_char_p, []),
    ("kmh_ctx_create", _c.c_int, [_c.c_int, _c.POINTER(_vp)]),
    ("kmh_ctx_destroy", None, [_vp]),
    ("kmh_ctx_release", _c.c_int, [_vp]),
    ("kmh_ctx_workspace_bytes", _u64, [_vp]),
    ("kmh_ctx_trim", _c.c_int, [_vp, _u64]),
    ("kmh_ctx_stats", _c.c_int, [_vp, _vp, _c.c_int]),
    ("kmh_last_error", _c.c_char_p, [_vp]),
    ("kmh_timing_enable", _c.c_int, [_vp, _c.c_int]),
    ("kmh_timing_report", _c.c_int, [_vp, _c.POINTER(_c.c_char_p), _u64p,
                                     _c.POINTER(_c.c_double), _c.c_int]),
    ("kmh_fasta_read", _c.c_int, [_c.c_char_p, _c.POINTER(_vp)]),
    ("kmh_fasta_count", _u64, [_vp]),
    ("kmh_fasta_record", _c.c_int, [_vp, _u64, _c.POINTER(_c.c_char_p), _u64p,
                                    _c.POINTER(_vp), _u64p, _u64p]),
    ("kmh_fasta_pack", _c.c_int, [_vp, _u64, _vp, _u64, _u64p, _vp]),
    ("kmh_fasta_free", None, [_vp]),
    ("kmh_count_host", _c.c_int, [_vp, _vp, _u64, _c.c_int, _c.c_int, _c.POINTER(_vp)]),
    ("kmh_stage_host", _c.c_int, [_vp, _vp, _u64]),
    ("kmh_count_staged", _c.c_int, [_vp, _c.c_int, _c.c_int, _c.POINTER(_vp)]),
    ("kmh_kmers_size", _u64, [_vp]),
    ("kmh_kmers_export", _c.c_int, [_vp, _vp, _vp, _vp]),
    ("kmh_kmers_data", _c.c_int, [_vp, _vp, _vp, _vp]),
    ("kmh_kmers_free", None, [_vp]),
    ("kmh_count_dense_host", _c.c_int, [_vp, _vp, _u64, _c.c_int, _vp]),
    ("kmh_count_dense_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _vp, _vp]),
    ("kmh_first_dense_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _vp, _vp]),
    ("kmh_synth_dev", _c.c_int, [_vp, _vp, _u64, _u64, _c.c_int, _u64, _vp]),
    ("kmh_format_lines", _c.c_int64, [_c.c_int, _vp, _vp, _u64, _vp, _u64]),
    ("kmh_format_lines_seq", _c.c_int64, [_c.c_int, _vp, _u64, _vp, _vp, _u64, _vp, _u64]),
    ("kmh_write_file", _c.c_int, [_c.c_char_p, _vp, _u64, _c.c_int, _c.c_int]),
    ("kmh_count_sparse_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _c.c_int, _vp, _vp, _vp, _vp]),
    ("kmh_count_sparse_sorted_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _c.c_int, _vp, _vp, _vp, _vp,
                                               _vp]),
    ("kmh_shard_union_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _u64, _u64, _vp, _vp, _u64p, _vp]),
    ("kmh_shard_union_u32_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _u64, _u64, _vp, _vp, _u64p, _vp]),
    ("kmh_rows_cuts_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _vp, _c.c_int, _vp, _vp]),
    ("kmh_wire_size_dev", _c.c_int, [_vp, _vp, _vp, _vp, _vp, _c.c_int, _vp, _vp]),
    ("kmh_wire_encode_dev", _c.c_int, [_vp, _vp, _vp, _vp, _vp, _c.c_int, _vp, _u64, _vp]),
    ("kmh_wire_decode_dev", _c.c_int, [_vp, _vp, _u64, _vp, _vp, _vp, _c.c_int, _vp, _vp, _vp]),
    ("kmh_sparse_out_offsets", _u64, [_vp, _c.c_int, _c.c_int, _vp]),
    ("kmh_rows_encode_u8_dev", _c.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _c.c_uint32, _vp, _vp]),
    ("kmh_rows_encode_u4_dev", _c.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _c.c_uint32, _vp, _vp]),
    ("kmh_rows_decode_u4_dev", _c.c_int, [_vp, _vp, _u64, _u64, _vp, _c.c_uint32, _vp, _vp, _vp]),
    ("kmh_count_dense_u4_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _vp, _vp, _vp, _c.c_uint32, _vp,
                                          _vp]),
    ("kmh_count_dense_u4only_dev", _c.c_int, [_vp, _vp, _vp, _c.c_int, _c.c_int, _vp, _vp, _vp, _c.c_uint32,
                                              _vp, _vp]),
    ("kmh_rows_decode_u4_range_dev", _c.c_int, [_vp, _vp, _u64, _u64, _vp, _c.c_uint32, _vp, _u64, _u64,
                                                _vp, _vp]),
    ("kmh_rows_decode_u8_dev", _c.c_int, [_vp, _vp, _u64, _u64, _vp, _c.c_uint32, _vp, _c.c_int,
                                          _u64, _vp, _vp]),
    ("kmh_feature_columns_dev", _c.c_int, [_vp, _vp, _u64, _c.c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("kmh_csv_format", _c.c_int, [_c.c_int, _vp, _vp, _vp, _u64, _c.c_int, _c.POINTER(_vp)]),
    ("kmh_text_data", _c.c_int, [_vp, _c.POINTER(_vp), _u64p]),
    ("kmh_text_free", None, [_vp]),
]

CSV_I64, CSV_F64, CSV_STR, CSV_LABEL, CSV_U64 = 0, 1, 2, 3, 4

_lib = None
_lib_lock = threading.Lock()
_ctx_lock = threading.Lock()   # separate: context() loads the library while holding it
_contexts = {}


class KmhError(RuntimeError):
    """A libkmerhip call failed; ``code`` is the KMH_ERR_* value."""

    def __init__(self, code, message):
        super().__init__(f"libkmerhip error {code}: {message}")
        self.code = code


def lib():
    """Load libkmerhip.so (raises ImportError if it was not built)."""
    global _lib
    if _lib is None:
        with _lib_lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"libkmerhip.so not found at {LIB_PATH}; build it with `make lib` "
                                      "(the k-mer path has no CPU fallback)")
                L = ctypes.CDLL(LIB_PATH)
                for name, res, args in SIGNATURES:
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                if LIB_PATH != DEFAULT_LIB_PATH:
                    import warnings
                    warnings.warn(f"KMH_LIB_PATH: using {LIB_PATH} (build {L.kmh_build_id().decode()}, "
                                  f"{L.kmh_version().decode()}) instead of the in-tree library")
                _lib = L
    return _lib


def build_id():
    """Source hash the loaded library was built from (kmh_build_id)."""
    return lib().kmh_build_id().decode()


def _check(rc, ctx=None):
    if rc < 0:
        msg = lib().kmh_last_error(ctx)
        msg = msg.decode(errors="replace") if msg else ""
        if rc == KMH_ERR_UNSUPPORTED:
            raise NotImplementedError(msg)
        if rc == KMH_ERR_INVALID:
            raise ValueError(msg)
        if rc == KMH_ERR_IO:
            raise OSError(msg)
        if rc == KMH_ERR_NOMEM:
            raise MemoryError(msg)
        raise KmhError(rc, msg)
    return rc


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _locked(fn):
    """Run a Context method under the context's lock: the C ABI serialises nothing itself, and
    release() / trim() free buffers that a call in flight on another thread would still use."""
    def wrapper(self, *args, **kwargs):
        with self.lock:
            return fn(self, *args, **kwargs)
    wrapper.__name__, wrapper.__doc__ = fn.__name__, fn.__doc__
    return wrapper


class Context:
    """A libkmerhip context bound to one HIP device (kmh_ctx_create).  Every call takes
    ``self.lock`` (re-entrant; hold it across kmh_stage_host + kmh_count_staged)."""

    def __init__(self, device=0):
        self.device = int(device)
        self.lock = threading.RLock()
        h = ctypes.c_void_p()
        _check(lib().kmh_ctx_create(self.device, ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    @_locked
    def close(self):
        if self._h:
            lib().kmh_ctx_destroy(self._h)
            self._h = None

    @_locked
    def release(self):
        """Free the cached device workspace (kmh_ctx_release); the next call allocates again."""
        if self._h:
            _check(lib().kmh_ctx_release(self._h), self._h)

    @_locked
    def workspace_bytes(self):
        """Device workspace + pinned staging the context holds now (kmh_ctx_workspace_bytes)."""
        return int(lib().kmh_ctx_workspace_bytes(self._h)) if self._h else 0

    @_locked
    def stats(self):
        """kmh_ctx_stats: {"fallback_passes", "fallback_groups", "workspace_bytes"}."""
        out = np.zeros(3, np.uint64)
        _check(lib().kmh_ctx_stats(self._h, _ptr(out), 3), self._h)
        return {"fallback_passes": int(out[0]), "fallback_groups": int(out[1]), "workspace_bytes": int(out[2])}

    @_locked
    def trim(self, keep_bytes):
        """kmh_ctx_trim: release the workspace if it holds more than keep_bytes."""
        if self._h:
            _check(lib().kmh_ctx_trim(self._h, int(keep_bytes)), self._h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-buffer counting (the drop-in path) --
    @_locked
    def count(self, seq, k, canonical=False):
        """Distinct k-mers of ``seq`` in first-occurrence order.

        Returns (codes u64, counts u32, first u64) numpy arrays; codes use A0 C1 G2 T3,
        first base most significant.
        """
        buf = _as_u8(seq)
        r = ctypes.c_void_p()
        _check(lib().kmh_count_host(self._h, _ptr(buf), buf.size, int(k), int(bool(canonical)),
                                    ctypes.byref(r)), self._h)
        return _kmers_arrays(r)

    @_locked
    def stage(self, seq):
        """kmh_stage_host: copy ``seq`` to the device once for several count_staged calls."""
        buf = _as_u8(seq)
        _check(lib().kmh_stage_host(self._h, _ptr(buf), buf.size), self._h)

    @_locked
    def count_staged(self, k, canonical=False):
        """count() of the sequence given to stage() (no second host-to-device copy)."""
        r = ctypes.c_void_p()
        _check(lib().kmh_count_staged(self._h, int(k), int(bool(canonical)), ctypes.byref(r)), self._h)
        return _kmers_arrays(r)

    @_locked
    def count_dense(self, seq, k):
        buf = _as_u8(seq)
        out = np.empty(1 << (2 * int(k)), np.uint32)
        _check(lib().kmh_count_dense_host(self._h, _ptr(buf), buf.size, int(k), _ptr(out)), self._h)
        return out


    # -- device-resident batch (pointers are device addresses, e.g. tensor.data_ptr()) --
    @_locked
    def count_dense_dev(self, d_seq, offsets, k, d_matrix, stream=None):
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        _check(lib().kmh_count_dense_dev(self._h, ctypes.c_void_p(d_seq), _ptr(off), off.size - 1,
                                         int(k), ctypes.c_void_p(d_matrix),
                                         ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def count_dense_u4_dev(self, d_seq, offsets, k, d_matrix, d_u4, d_esc, cap, d_esc_n, stream=None,
                           rows=True):
        """Count + u4 slot in one pass.  rows=False (kmh_count_dense_u4only_dev): d_matrix is
        scratch, not left holding the u32 rows."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        fn = lib().kmh_count_dense_u4_dev if rows else lib().kmh_count_dense_u4only_dev
        _check(fn(self._h, ctypes.c_void_p(d_seq), _ptr(off), off.size - 1, int(k), ctypes.c_void_p(d_matrix),
                  ctypes.c_void_p(d_u4), ctypes.c_void_p(d_esc), int(cap), ctypes.c_void_p(d_esc_n),
                  ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def first_dense_dev(self, d_seq, offsets, k, d_first, stream=None):
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        _check(lib().kmh_first_dense_dev(self._h, ctypes.c_void_p(d_seq), _ptr(off), off.size - 1,
                                         int(k), ctypes.c_void_p(d_first),
                                         ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def synth_dev(self, d_seq, length, stride, n_genomes, seed0, stream=None):
        _check(lib().kmh_synth_dev(self._h, ctypes.c_void_p(d_seq), int(length), int(stride),
                                   int(n_genomes), int(seed0),
                                   ctypes.c_void_p(stream) if stream else None), self._h)

    # -- sparse counting, device-resident (BASELINE config 5) --
    @_locked
    def count_sparse_dev(self, d_seq, offsets, k, canonical, d_codes, d_counts, d_nkmers, stream=None):
        """Distinct k-mers of G device-resident genomes (13 <= k <= 32); genome g's entries
        start at sparse_out_offsets(offsets, k)[g].  Synchronises the stream."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        _check(lib().kmh_count_sparse_dev(self._h, ctypes.c_void_p(d_seq), _ptr(off), off.size - 1, int(k),
                                          int(bool(canonical)), ctypes.c_void_p(d_codes),
                                          ctypes.c_void_p(d_counts), ctypes.c_void_p(d_nkmers),
                                          ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def count_sparse_sorted_dev(self, d_seq, offsets, k, canonical, d_codes, d_counts, d_nrows, d_ndistinct,
                                stream=None):
        """count_sparse_dev with every genome's rows in ascending code order (kmh_count_sparse_sorted_dev):
        the genomes' rows are back to back from entry 0 (genome g's after rows 0 .. g - 1), strictly
        ascending; d_nrows[g] = d_ndistinct[g] = its distinct k-mers.  Synchronises the stream."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        _check(lib().kmh_count_sparse_sorted_dev(self._h, ctypes.c_void_p(d_seq), _ptr(off), off.size - 1, int(k),
                                                 int(bool(canonical)), ctypes.c_void_p(d_codes),
                                                 ctypes.c_void_p(d_counts), ctypes.c_void_p(d_nrows),
                                                 ctypes.c_void_p(d_ndistinct),
                                                 ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def shard_union_dev(self, d_codes, row_off, lo_code, hi_code_incl, d_columns, d_indices, stream=None,
                        idx32=False):
        """kmh_shard_union_dev: the sorted union of R sorted rows (row r = d_codes[row_off[r],
        row_off[r + 1]), host offsets) into d_columns and every entry's column into d_indices
        (int64, or u32 with idx32=True: kmh_shard_union_u32_dev); returns the union's size."""
        ro = np.ascontiguousarray(row_off, dtype=np.uint64)
        n = ctypes.c_uint64(0)
        fn = lib().kmh_shard_union_u32_dev if idx32 else lib().kmh_shard_union_dev
        _check(fn(self._h, ctypes.c_void_p(d_codes), _ptr(ro), ro.size - 1, int(lo_code), int(hi_code_incl),
                  ctypes.c_void_p(d_columns), ctypes.c_void_p(d_indices), ctypes.byref(n),
                  ctypes.c_void_p(stream) if stream else None), self._h)
        return int(n.value)

    # -- the config-5 exchange (kmh_wire.hip) --
    @_locked
    def rows_cuts_dev(self, d_codes, row_off, bounds, d_cuts, stream=None):
        """kmh_rows_cuts_dev: d_cuts[r * nb + b] (device u64) = the first entry of sorted row r (host
        row_off) whose code is >= bounds[b] (host uint64 array)."""
        ro = np.ascontiguousarray(row_off, dtype=np.uint64)
        b = np.ascontiguousarray(bounds, dtype=np.uint64)
        _check(lib().kmh_rows_cuts_dev(self._h, ctypes.c_void_p(d_codes), _ptr(ro), ro.size - 1, _ptr(b), b.size,
                                       ctypes.c_void_p(d_cuts), ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def wire_size_dev(self, d_codes, d_counts, slice_start, slice_n, stream=None):
        """kmh_wire_size_dev: bytes of every slice in the compact wire format (uint64 array)."""
        st = np.ascontiguousarray(slice_start, dtype=np.uint64)
        sn = np.ascontiguousarray(slice_n, dtype=np.uint64)
        out = np.zeros(st.size, np.uint64)
        _check(lib().kmh_wire_size_dev(self._h, ctypes.c_void_p(d_codes), ctypes.c_void_p(d_counts), _ptr(st), _ptr(sn),
                                       st.size, _ptr(out), ctypes.c_void_p(stream) if stream else None), self._h)
        return out

    @_locked
    def wire_encode_dev(self, d_codes, d_counts, slice_start, slice_n, d_out, out_bytes, stream=None):
        """kmh_wire_encode_dev: the slices back to back at d_out (device)."""
        st = np.ascontiguousarray(slice_start, dtype=np.uint64)
        sn = np.ascontiguousarray(slice_n, dtype=np.uint64)
        _check(lib().kmh_wire_encode_dev(self._h, ctypes.c_void_p(d_codes), ctypes.c_void_p(d_counts), _ptr(st),
                                         _ptr(sn), st.size, ctypes.c_void_p(d_out), int(out_bytes),
                                         ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def wire_decode_dev(self, d_in, in_bytes, slice_n, slice_bytes, slice_dst, d_codes, d_counts, stream=None):
        """kmh_wire_decode_dev: slices back to back at d_in -> entries slice_dst[i] .. of d_codes / d_counts."""
        sn = np.ascontiguousarray(slice_n, dtype=np.uint64)
        sb = np.ascontiguousarray(slice_bytes, dtype=np.uint64)
        sd = np.ascontiguousarray(slice_dst, dtype=np.uint64)
        _check(lib().kmh_wire_decode_dev(self._h, ctypes.c_void_p(d_in), int(in_bytes), _ptr(sn), _ptr(sb), _ptr(sd),
                                         sn.size, ctypes.c_void_p(d_codes), ctypes.c_void_p(d_counts),
                                         ctypes.c_void_p(stream) if stream else None), self._h)

    # -- matrix assembly encoding (device pointers) --
    @_locked
    def rows_encode_u8(self, d_rows, rows, cols, d_u8, d_esc, cap, d_esc_n, stream=None):
        _check(lib().kmh_rows_encode_u8_dev(self._h, ctypes.c_void_p(d_rows), int(rows), int(cols),
                                            ctypes.c_void_p(d_u8), ctypes.c_void_p(d_esc), int(cap),
                                            ctypes.c_void_p(d_esc_n),
                                            ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def rows_decode_u8(self, d_u8, rows, cols, d_esc, cap, d_esc_n, ranks, rows_per_rank, d_rows,
                       stream=None):
        _check(lib().kmh_rows_decode_u8_dev(self._h, ctypes.c_void_p(d_u8), int(rows), int(cols),
                                            ctypes.c_void_p(d_esc), int(cap), ctypes.c_void_p(d_esc_n),
                                            int(ranks), int(rows_per_rank), ctypes.c_void_p(d_rows),
                                            ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def rows_encode_u4(self, d_rows, rows, cols, d_u4, d_esc, cap, d_esc_n, stream=None):
        _check(lib().kmh_rows_encode_u4_dev(self._h, ctypes.c_void_p(d_rows), int(rows), int(cols),
                                            ctypes.c_void_p(d_u4), ctypes.c_void_p(d_esc), int(cap),
                                            ctypes.c_void_p(d_esc_n),
                                            ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def rows_decode_u4(self, d_u4, rows, cols, d_esc, cap, d_esc_n, d_rows, stream=None):
        _check(lib().kmh_rows_decode_u4_dev(self._h, ctypes.c_void_p(d_u4), int(rows), int(cols),
                                            ctypes.c_void_p(d_esc), int(cap), ctypes.c_void_p(d_esc_n),
                                            ctypes.c_void_p(d_rows),
                                            ctypes.c_void_p(stream) if stream else None), self._h)

    @_locked
    def rows_decode_u4_range(self, d_u4, rows, cols, d_esc, cap, d_esc_n, row0, nrows, d_rows, stream=None):
        _check(lib().kmh_rows_decode_u4_range_dev(self._h, ctypes.c_void_p(d_u4), int(rows), int(cols),
                                                  ctypes.c_void_p(d_esc), int(cap), ctypes.c_void_p(d_esc_n),
                                                  int(row0), int(nrows), ctypes.c_void_p(d_rows),
                                                  ctypes.c_void_p(stream) if stream else None), self._h)

    # -- feature columns (device pointers; statistics.py:188-238) --
    @_locked
    def feature_columns_dev(self, d_codes, n, k, d_order, d_lg, d_cnt, d_cpg, d_rep, d_gc, d_oe, d_ent, stream=None):
        _check(lib().kmh_feature_columns_dev(self._h, ctypes.c_void_p(d_codes) if d_codes else None, int(n), int(k),
                                             ctypes.c_void_p(d_order), ctypes.c_void_p(d_lg), ctypes.c_void_p(d_cnt),
                                             ctypes.c_void_p(d_cpg), ctypes.c_void_p(d_rep), ctypes.c_void_p(d_gc),
                                             ctypes.c_void_p(d_oe), ctypes.c_void_p(d_ent),
                                             ctypes.c_void_p(stream) if stream else None), self._h)

    # -- kernel timing --
    @_locked
    def timing(self, enable):
        _check(lib().kmh_timing_enable(self._h, int(bool(enable))), self._h)

    @_locked
    def timing_report(self):
        cap = 64
        names = (ctypes.c_char_p * cap)()
        launches = (ctypes.c_uint64 * cap)()
        total = (ctypes.c_double * cap)()
        n = _check(lib().kmh_timing_report(self._h, names, launches, total, cap), self._h)
        return {names[i].decode(): (int(launches[i]), float(total[i])) for i in range(min(n, cap))}


def context(device=0):
    """Process-wide context per device (created on first use)."""
    device = int(device)
    with _ctx_lock:
        ctx = _contexts.get(device)
        if ctx is None:
            ctx = Context(device)
            _contexts[device] = ctx
    return ctx


def release_all():
    """kmh_ctx_release on every process-wide context (before handing the GPU to other
    processes, e.g. ranks started on the same device)."""
    with _ctx_lock:
        ctxs = list(_contexts.values())
    for c in ctxs:
        c.release()


def _as_u8(seq):
    if isinstance(seq, np.ndarray):
        return np.ascontiguousarray(seq, dtype=np.uint8)
    return np.frombuffer(bytes(seq), dtype=np.uint8)


def _kmers_arrays(r):
    """(codes u64, counts u32, first u64) numpy views of a kmh_kmers result (no copy; the views
    keep the result alive)."""
    owner = _Kmers(r)
    n = lib().kmh_kmers_size(r)
    if n == 0:
        return np.empty(0, np.uint64), np.empty(0, np.uint32), np.empty(0, np.uint64)
    pc, pn, pf = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    _check(lib().kmh_kmers_data(r, ctypes.byref(pc), ctypes.byref(pn), ctypes.byref(pf)))
    return (owner.view(pc, n, ctypes.c_uint64), owner.view(pn, n, ctypes.c_uint32),
            owner.view(pf, n, ctypes.c_uint64))


class _Kmers:
    """Owns a kmh_kmers result; numpy views of its arrays keep it alive through their base
    (a ctypes array over the C memory that holds a reference to this object)."""

    def __init__(self, handle):
        self._h = handle

    def view(self, ptr, n, ctype):
        buf = (ctype * n).from_address(ptr.value)
        buf._owner = self
        return np.frombuffer(buf, dtype=np.dtype(ctype))

    def __del__(self):
        if self._h:
            lib().kmh_kmers_free(self._h)
            self._h = None


class FastaFile:
    """Records of a FASTA file parsed by kmh_fasta_read (generate.py:39-41 semantics)."""

    def __init__(self, path):
        h = ctypes.c_void_p()
        _check(lib().kmh_fasta_read(os.fsencode(str(path)), ctypes.byref(h)))
        self._h = h
        n = lib().kmh_fasta_count(h)
        self.ids, self.char_lens, self.seq_lens = [], [], []
        idp, idl = ctypes.c_char_p(), ctypes.c_uint64()
        sp, sl, cl = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
        for i in range(n):
            _check(lib().kmh_fasta_record(h, i, ctypes.byref(idp), ctypes.byref(idl),
                                          ctypes.byref(sp), ctypes.byref(sl), ctypes.byref(cl)))
            raw = ctypes.string_at(idp, idl.value) if idl.value else b""
            self.ids.append(raw.decode("utf-8", errors="surrogateescape"))
            self.seq_lens.append(sl.value)
            self.char_lens.append(cl.value)

    def __len__(self):
        return len(self.ids)

    def sequence(self, i):
        sp, sl = ctypes.c_void_p(), ctypes.c_uint64()
        _check(lib().kmh_fasta_record(self._h, i, None, None, ctypes.byref(sp), ctypes.byref(sl), None))
        return ctypes.string_at(sp, sl.value) if sl.value else b""

    def pack(self, min_len, align=1):
        """Kept records (char length >= min_len) joined by '\\n' -> (uint8 array, kept flags).

        Records with multi-byte UTF-8 characters go through Python's own str.upper() first
        (generate.py:41 upper-cases before the length rule of :44): a few code points expand
        (U+00DF -> "SS" lengthens the record; U+FB05 / U+FB06 -> "ST", U+1E97 -> "T" + U+0308 and
        U+1E9A -> "A" + U+02BE put bases into it); every non-ASCII character of the result is
        then written as '?', a non-base.  ASCII records are packed by kmh_fasta_pack (the
        kernels fold their case)."""
        if any(c != n for c, n in zip(self.char_lens, self.seq_lens)):
            return self._pack_unicode(min_len, align)
        need = ctypes.c_uint64()
        kept = np.zeros(max(len(self), 1), np.uint8)
        _check(lib().kmh_fasta_pack(self._h, int(min_len), None, 0, ctypes.byref(need), _ptr(kept)))
        out = np.empty(need.value + align, np.uint8)
        _check(lib().kmh_fasta_pack(self._h, int(min_len), _ptr(out), out.size, ctypes.byref(need),
                                    None))
        return out[:need.value], kept[:len(self)].astype(bool)

    def _pack_unicode(self, min_len, align):
        parts, kept = [], np.zeros(len(self), bool)
        for i in range(len(self)):
            raw = self.sequence(i)
            if self.char_lens[i] == self.seq_lens[i]:
                n, body = self.char_lens[i], raw
            else:
                up = raw.decode("utf-8", errors="surrogateescape").upper()
                n, body = len(up), up.encode("ascii", errors="replace")
            if n >= min_len:
                kept[i] = True
                parts.append(body)
        data = b"\n".join(parts)
        out = np.empty(len(data) + align, np.uint8)
        out[:len(data)] = np.frombuffer(data, np.uint8)
        return out[:len(data)], kept

    def close(self):
        if self._h:
            lib().kmh_fasta_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_file(path, data, gzip_level=-1, threads=0):
    """Write bytes to path (gzip_level 0..9: multi-member gzip deflated on several threads)."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    _check(lib().kmh_write_file(os.fsencode(str(path)), _ptr(buf), len(data), int(gzip_level), int(threads)))


def format_lines_array(k, codes, counts):
    """k{k}.txt text for (codes, counts) -- generate.py:86-91 -- as a uint8 array (written
    in place: no zero-filled staging buffer, no copy into a bytes object)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint64)
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    n = codes.size
    need = _check(lib().kmh_format_lines(int(k), _ptr(codes), _ptr(counts), n, None, 0))
    out = np.empty(max(need, 1), np.uint8)
    _check(lib().kmh_format_lines(int(k), _ptr(codes), _ptr(counts), n, _ptr(out), need))
    return out[:need]


def format_lines(k, codes, counts):
    """k{k}.txt bytes for (codes, counts) -- generate.py:86-91 text."""
    return format_lines_array(k, codes, counts).tobytes()


def format_lines_seq(k, seq, first, counts):
    """k{k}.txt bytes for any k, the digits of line i taken from seq[first[i] : first[i] + k]
    (``seq`` = the buffer the k-mers were counted in; the form used for k > 32)."""
    buf = _as_u8(seq)
    first = np.ascontiguousarray(first, dtype=np.uint64)
    counts = np.ascontiguousarray(counts, dtype=np.uint64)
    n = first.size
    need = _check(lib().kmh_format_lines_seq(int(k), _ptr(buf), buf.size, _ptr(first), _ptr(counts), n, None, 0))
    out = ctypes.create_string_buffer(max(need, 1))
    _check(lib().kmh_format_lines_seq(int(k), _ptr(buf), buf.size, _ptr(first), _ptr(counts), n, out, need))
    return out.raw[:need]


def sparse_out_offsets(offsets, k):
    """Entry offsets of every genome in the output of Context.count_sparse_dev (G + 1)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = np.zeros(off.size, dtype=np.uint64)
    lib().kmh_sparse_out_offsets(_ptr(off), off.size - 1, int(k), _ptr(out))
    return out


class _Text:
    """Owns a kmh_text; the numpy view of its bytes keeps it alive."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if self._h:
            lib().kmh_text_free(self._h)
            self._h = None


def csv_format(columns, nrows, threads=0):
    """CSV rows of a column block (kmh_csv_format: pandas' to_csv text without the header).

    columns: list of (kind, data, aux) with kind one of CSV_*: CSV_I64 / CSV_U64 / CSV_F64 take a
    numpy array; CSV_STR a (utf-8 bytes, uint64 offsets[nrows + 1]) pair as (data, aux); CSV_LABEL
    uint64 codes and aux = k.  Returns a uint8 numpy view of the text (no copy), or None when
    pandas would write some value differently (NaN / inf, text needing quotes)."""
    keep = []
    kinds = np.array([c[0] for c in columns], dtype=np.int32)
    data = (ctypes.c_void_p * max(len(columns), 1))()
    aux = (ctypes.c_void_p * max(len(columns), 1))()
    for j, (kind, d, x) in enumerate(columns):
        if kind in (CSV_I64, CSV_U64, CSV_F64):
            arr = np.ascontiguousarray(d, dtype={CSV_I64: np.int64, CSV_U64: np.uint64, CSV_F64: np.float64}[kind])
            keep.append(arr)
            data[j] = arr.ctypes.data if arr.size else None
        elif kind == CSV_STR:
            buf = np.frombuffer(d, np.uint8) if len(d) else np.zeros(1, np.uint8)
            off = np.ascontiguousarray(x, dtype=np.uint64)
            keep += [buf, off]
            data[j], aux[j] = buf.ctypes.data, off.ctypes.data
        elif kind == CSV_LABEL:
            arr = np.ascontiguousarray(d, dtype=np.uint64)
            kk = np.array([int(x)], dtype=np.int64)
            keep += [arr, kk]
            data[j], aux[j] = (arr.ctypes.data if arr.size else None), kk.ctypes.data
        else:
            raise ValueError(f"csv_format: unknown column kind {kind}")
    h = ctypes.c_void_p()
    rc = lib().kmh_csv_format(len(columns), _ptr(kinds), data, aux, int(nrows), int(threads), ctypes.byref(h))
    if rc == KMH_ERR_UNSUPPORTED:
        return None
    _check(rc)
    owner = _Text(h)
    p, n = ctypes.c_void_p(), ctypes.c_uint64()
    _check(lib().kmh_text_data(h, ctypes.byref(p), ctypes.byref(n)))
    if n.value == 0:
        return np.zeros(0, np.uint8)
    buf = (ctypes.c_uint8 * n.value).from_address(p.value)
    buf._owner = owner
    return np.frombuffer(buf, dtype=np.uint8)
