"""ctypes binding of libcc_mi355x.so (the C ABI in include/cc_mi355x.h).

This is the only way the product reaches the GPU.  There is no CPU fallback: if the
library is missing or no GPU is visible, every compute call raises.

Arrays: host numpy arrays go through the *_host entry points; device buffers are
torch CUDA tensors (ROCm) passed by data_ptr().
"""
import ctypes
import os
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('CC_LIB_PATH') or os.path.join(_HERE, 'lib', 'libcc_mi355x.so')   # override: A/B timing only
MODES = {'greater': 0, 'less': 1, 'equal': 2}

# every symbol include/cc_mi355x.h declares (checked by tests/test_boundary.py)
EXPORTS = (
    'cc_create', 'cc_destroy', 'cc_last_error', 'cc_set_stream', 'cc_version',
    'cc_label_volume', 'cc_label_volume_host', 'cc_get_block_values', 'cc_get_offsets',
    'cc_get_lut', 'cc_block_components', 'cc_merge_offsets', 'cc_block_faces',
    'cc_merge_assignments', 'cc_write', 'cc_generate_boundary_map', 'cc_set_profiling',
    'cc_get_profile', 'cc_reset_profile', 'cc_shard_begin', 'cc_shard_assign', 'cc_shard_planes',
    'cc_seam_pairs', 'cc_shard_finish', 'cc_set_debug', 'cc_threshold', 'cc_shard_top_plane32',
    'cc_seam_pairs32', 'cc_shard_top_cubes32', 'cc_seam_pairs_cubes32',
    'cc_evaluate', 'cc_get_overlaps', 'cc_relabel_consecutive', 'cc_set_option', 'cc_channel_mean',
    'cc_gaussian_smooth_blocks', 'cc_gaussian_taps', 'cc_result_size', 'cc_resize_mask_nearest',
    'cc_watershed_from_seeds', 'cc_shard_dev_begin', 'cc_shard_dev_assign', 'cc_shard_dev_top_cubes',
    'cc_shard_dev_seam_pairs', 'cc_shard_dev_finish', 'cc_normalize_channels', 'cc_shard_dev_ok',
    'cc_comm_unique_id', 'cc_comm_create', 'cc_comm_destroy', 'cc_label_volume_sharded', 'cc_comm_info',
)
# redo flags of the one-read-back schedule (RF_* in csrc/cc_kernels.hip)
RF_BIG, RF_ROOTS, RF_CUBES, RF_PAIRS, RF_IOVF = 1, 2, 4, 8, 16
CC_ERR_ID_RANGE = -3          # cc_evaluate: ids beyond the key packing (include/cc_mi355x.h)
# CC_DTYPE_* of include/cc_mi355x.h (cc_channel_mean)
DTYPES = {'float32': 0, 'float64': 1, 'uint8': 2, 'int8': 3, 'uint16': 4, 'int16': 5, 'uint32': 6,
          'int32': 7, 'uint64': 8, 'int64': 9}
# every symbol include/cc_n5.h declares (libcc_n5.so: host-only N5 codec)
# override: the sanitizer build (tools/asan.sh) only
N5_LIB_PATH = os.environ.get('CC_N5_LIB_PATH') or os.path.join(_HERE, 'lib', 'libcc_n5.so')
N5_EXPORTS = ('cc_n5_version', 'cc_n5_last_error', 'cc_n5_read', 'cc_n5_write')


class CCResult(ctypes.Structure):
    _fields_ = [('n_blocks', ctypes.c_int64), ('n_labels', ctypes.c_uint64),
                ('max_id', ctypes.c_uint64), ('n_components', ctypes.c_uint64),
                ('n_block_components', ctypes.c_uint64), ('n_relabelled_tiles', ctypes.c_uint64),
                ('identity_lut', ctypes.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class CCEvalResult(ctypes.Structure):
    _fields_ = [('n_points', ctypes.c_uint64), ('n_pairs', ctypes.c_uint64),
                ('n_seg_ids', ctypes.c_uint64), ('n_gt_ids', ctypes.c_uint64),
                ('vi_split', ctypes.c_double), ('vi_merge', ctypes.c_double),
                ('adapted_rand_error', ctypes.c_double), ('rand_index', ctypes.c_double),
                ('sum_sq_pairs', ctypes.c_double), ('sum_sq_gt', ctypes.c_double),
                ('sum_sq_seg', ctypes.c_double)]

    def as_dict(self):
        return {k: (float if t is ctypes.c_double else int)(getattr(self, k)) for k, t in self._fields_}


_lib = None
_host_only = False


def load(host_only=False):
    """Load the shared library and declare signatures (no GPU needed).

    One HIP runtime per process: torch bundles its own libamdhip64 (SONAME libamdhip64.so.7), and
    the library must bind to that one.  Loaded first, the library would pull /opt/rocm's copy and
    torch would then load a second runtime beside it (the second to initialise sees no device), so
    torch is imported first.  host_only=True is for processes that never touch torch (the drop-in's
    job processes on numpy buffers: cc_label_volume_host, cc_merge_offsets): without torch already
    imported, the library binds the system HIP runtime and the ~2 s torch import is skipped; a later
    import of torch in such a process is refused here."""
    global _lib, _host_only
    if _lib is not None:
        if _host_only and not host_only and 'torch' in sys.modules:
            raise RuntimeError('libcc_mi355x.so was loaded host-only (without torch) in this process; '
                               'torch tensors cannot be used with it here')
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('libcc_mi355x.so not built (%s): run __graft_entry__.build()' % LIB_PATH)
    if host_only and 'torch' not in sys.modules:
        _host_only = True
    else:
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(LIB_PATH)
    P, i64, u64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_int
    sig = {
        'cc_create': (I, [I, ctypes.POINTER(P)]),
        'cc_destroy': (None, [P]),
        'cc_last_error': (ctypes.c_char_p, []),
        'cc_set_stream': (I, [P, P]),
        'cc_version': (ctypes.c_char_p, []),
        'cc_label_volume': (I, [P, P, P, P, P, ctypes.c_double, I, P, ctypes.POINTER(CCResult)]),
        'cc_label_volume_host': (I, [P, P, P, P, P, ctypes.c_double, I, P, ctypes.POINTER(CCResult)]),
        'cc_get_block_values': (i64, [P, P, i64]),
        'cc_get_offsets': (i64, [P, P, i64]),
        'cc_get_lut': (i64, [P, P, i64]),
        'cc_block_components': (I, [P, P, P, P, P, ctypes.c_double, I, P, P, i64]),
        'cc_merge_offsets': (I, [P, i64, P, P, P]),
        'cc_block_faces': (i64, [P, P, P, P, P, P, i64, P]),
        'cc_set_option': (I, [P, I, i64]),
        'cc_merge_assignments': (I, [P, P, i64, u64, P]),
        'cc_write': (I, [P, P, P, P, P, P, u64]),
        'cc_generate_boundary_map': (I, [P, P, P, P, u64, I]),
        'cc_set_profiling': (I, [P, I]),
        'cc_get_profile': (I, [P, ctypes.c_char_p, I, P, P, I]),
        'cc_reset_profile': (I, [P]),
        'cc_set_debug': (I, [P, I]),
        'cc_threshold': (I, [P, P, P, P, ctypes.c_double, I, P]),
        'cc_shard_top_plane32': (I, [P, P]),
        'cc_seam_pairs32': (i64, [P, P, u64, P, i64, P, i64]),
        'cc_shard_top_cubes32': (I, [P, P]),
        'cc_seam_pairs_cubes32': (i64, [P, P, u64, P, i64, i64, P, i64]),
        'cc_shard_begin': (I, [P, P, P, P, P, ctypes.c_double, I, i64, P]),
        'cc_shard_assign': (I, [P, u64]),
        'cc_shard_planes': (I, [P, P, P]),
        'cc_seam_pairs': (i64, [P, P, P, i64, P, i64]),
        'cc_shard_finish': (I, [P, P, i64, P, ctypes.POINTER(CCResult)]),
        'cc_shard_dev_ok': (I, [P]),
        'cc_comm_unique_id': (I, [P, i64]),
        'cc_comm_create': (I, [P, I, I, I, ctypes.POINTER(P)]),
        'cc_comm_destroy': (None, [P]),
        'cc_comm_info': (I, [P, P]),
        'cc_label_volume_sharded': (I, [P, P, P, P, P, i64, i64, P, ctypes.c_double, I, P, ctypes.POINTER(CCResult)]),
        'cc_shard_dev_begin': (I, [P, P, P, P, P, ctypes.c_double, I, i64, P]),
        'cc_shard_dev_assign': (I, [P, P, I, I]),
        'cc_shard_dev_top_cubes': (I, [P, P]),
        'cc_shard_dev_seam_pairs': (I, [P, P, P, I, P, i64]),
        'cc_shard_dev_finish': (I, [P, P, I, i64, P, P, ctypes.POINTER(CCResult), P]),
        'cc_evaluate': (I, [P, P, P, P, P, I, u64, ctypes.POINTER(CCEvalResult)]),
        'cc_get_overlaps': (i64, [P, P, P, P, i64]),
        'cc_relabel_consecutive': (I, [P, P, P, i64, P, P, P, i64]),
        'cc_channel_mean': (I, [P, P, I, P, P, i64, P]),
        'cc_gaussian_smooth_blocks': (I, [P, P, P, P, ctypes.c_double, P]),
        'cc_gaussian_taps': (I, [ctypes.c_double, P, I]),
        'cc_result_size': (i64, []),
        'cc_resize_mask_nearest': (I, [P, P, P, P, i64, i64, P]),
        'cc_watershed_from_seeds': (I, [P, P, P, P, P, P, P, P]),
        'cc_normalize_channels': (I, [P, P, i64, P, P, I, P]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if os.environ.get('CC_LIB_PATH'):   # an older build for same-box A/B timing: newer entries absent
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


_n5 = None


def load_n5():
    """The host-only N5 codec library (no GPU runtime)."""
    global _n5
    if _n5 is not None:
        return _n5
    if not os.path.exists(N5_LIB_PATH):
        raise RuntimeError('libcc_n5.so not built (%s): run __graft_entry__.build()' % N5_LIB_PATH)
    L = ctypes.CDLL(N5_LIB_PATH)
    P, I = ctypes.c_void_p, ctypes.c_int
    sig = {
        'cc_n5_version': (ctypes.c_char_p, []),
        'cc_n5_last_error': (ctypes.c_char_p, []),
        'cc_n5_read': (I, [ctypes.c_char_p, I, P, P, I, I, P, P, P, I]),
        'cc_n5_write': (I, [ctypes.c_char_p, I, P, P, I, I, I, P, P, P, I, I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _n5 = L
    return L


def _check_n5(rc):
    if rc < 0:
        raise RuntimeError('libcc_n5: ' + load_n5().cc_n5_last_error().decode())
    return rc


def version():
    return load().cc_version().decode()


def gaussian_taps(sigma):
    """The 2r + 1 float32 taps of the sigma_prefilter kernel (cc_gaussian_taps)."""
    buf = np.zeros(129, dtype=np.float32)
    r = _check(load().cc_gaussian_taps(float(sigma), _ptr(buf), len(buf)))
    return buf[:2 * r + 1].copy()


def check_provenance():
    """Raise unless the loaded library was built from this tree's sources: cc_version()
    carries the SHA-256 prefix build.py embedded (binary provenance)."""
    from . import build
    want = build.source_hash()
    for path, v in ((LIB_PATH, version()), (N5_LIB_PATH, load_n5().cc_n5_version().decode())):
        got = v.split('src=')[-1] if 'src=' in v else None
        if got != want:
            raise RuntimeError('%s was built from other sources (library src=%s, tree src=%s): rebuild with '
                               '__graft_entry__.build()' % (path, got, want))
    return want


def _check(rc):
    if rc < 0:
        raise RuntimeError('libcc_mi355x: ' + load().cc_last_error().decode())
    return rc


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64))


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, 'data_ptr'):
        return a.data_ptr()
    return a.ctypes.data


def mode_id(mode):
    if isinstance(mode, int):
        return mode
    if mode not in MODES:
        raise ValueError('threshold_mode must be one of %s' % (tuple(MODES),))
    return MODES[mode]


def comm_unique_id():
    """The RCCL bootstrap id (128 bytes) for Comm: made on one rank, handed to every rank."""
    buf = ctypes.create_string_buffer(128)
    _check(load().cc_comm_unique_id(buf, 128))
    return buf.raw


class Comm:
    """One rank's RCCL communicator owned by the library (cc_comm_create): z-slab sharding from a
    plain C / ctypes caller, no torch.distributed (Context.label_volume_sharded)."""

    def __init__(self, unique_id, world, rank, device=0):
        h = ctypes.c_void_p()
        uid = ctypes.create_string_buffer(bytes(unique_id), 128)
        _check(load().cc_comm_create(uid, int(world), int(rank), int(device), ctypes.byref(h)))
        self._h, self.world, self.rank, self.device = h, world, rank, device

    def info(self):
        """cc_comm_info: world, rank, the last call's schedule ('one-read-back' / 'synchronised' /
        None), its redo flags (RF_*), the seam-pair capacity, whether an error aborted the
        communicator, and the number of calls."""
        out = (ctypes.c_int64 * 8)()
        _check(load().cc_comm_info(self._h, out))
        return {'world': out[0], 'rank': out[1],
                'schedule': {1: 'one-read-back', 0: 'synchronised'}.get(out[2]),
                'redo': out[3], 'pair_cap': out[4], 'aborted': bool(out[5]), 'calls': out[6]}

    def close(self):
        if self._h:
            load().cc_comm_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class Context:
    """One cc_ctx (one GPU).  Not thread-safe."""

    def __init__(self, device=0):
        L = load()
        h = ctypes.c_void_p()
        _check(L.cc_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if self._h:
            load().cc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_ptr):
        _check(load().cc_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None))
        self._stream = stream_ptr or None

    # ---- fused path ----
    def label_volume(self, inp, block_shape, threshold, mode='greater', mask=None, out=None):
        """Fused five-stage path.  `inp` is a float32 torch CUDA tensor (device path) or a
        numpy array (host path).  Returns (labels, result dict)."""
        L = load()
        shape = _i64(inp.shape)
        bs = _i64(block_shape)
        assert len(shape) == 3 and len(bs) == 3
        res = CCResult()
        if hasattr(inp, 'data_ptr'):
            import torch
            assert inp.is_cuda and inp.dtype == torch.float32 and inp.is_contiguous()
            if mask is not None:
                assert mask.is_cuda and mask.dtype == torch.uint8 and mask.shape == inp.shape
                mask = mask.contiguous()
            if out is None:
                out = torch.empty(tuple(inp.shape), dtype=torch.int64, device=inp.device)
            _check(L.cc_label_volume(self._h, _ptr(inp), _ptr(mask), _ptr(shape), _ptr(bs),
                                     float(threshold), mode_id(mode), _ptr(out), ctypes.byref(res)))
        else:
            inp = np.ascontiguousarray(inp, dtype=np.float32)
            if mask is not None:
                mask = np.ascontiguousarray(mask)
                if mask.dtype != np.uint8:
                    mask = (mask != 0).astype(np.uint8)
                assert mask.shape == inp.shape
            if out is None:
                out = np.empty(inp.shape, dtype=np.uint64)
            _check(L.cc_label_volume_host(self._h, _ptr(inp), _ptr(mask), _ptr(shape), _ptr(bs),
                                          float(threshold), mode_id(mode), _ptr(out), ctypes.byref(res)))
        return out, res.as_dict()

    def label_volume_sharded(self, comm, slab, global_shape, z_offset, block_shape, threshold, mode='greater',
                             mask=None, out=None):
        """This rank's z-slab [z_offset, z_offset + len(slab)) of a volume sharded over comm's ranks
        (cc_label_volume_sharded: the schedule with RCCL inside the library).  `slab` / `mask`:
        CUDA tensors of the slab.  Returns (labels of the slab, result dict with the global
        n_labels).  The call is collective (every rank of comm calls it).  It runs on the stream
        bound with set_stream if there is one; else it is ordered on torch's current stream: on the
        default (null) stream the library fences its own stream against it, another current stream
        is bound to the context for the call."""
        import torch
        assert slab.is_cuda and slab.dtype == torch.float32 and slab.is_contiguous() and slab.dim() == 3
        if mask is not None:
            assert mask.is_cuda and mask.dtype == torch.uint8 and mask.shape == slab.shape
            mask = mask.contiguous()
        if out is None:
            out = torch.empty(tuple(slab.shape), dtype=torch.int64, device=slab.device)
        gs, bs = _i64(global_shape), _i64(block_shape)
        res = CCResult()
        prev = getattr(self, '_stream', None)
        cur = prev or torch.cuda.current_stream(slab.device).cuda_stream or None
        if cur != prev:
            self.set_stream(cur)
        try:
            _check(load().cc_label_volume_sharded(self._h, comm._h, _ptr(slab), _ptr(mask), _ptr(gs), int(z_offset),
                                                  int(slab.shape[0]), _ptr(bs), float(threshold), mode_id(mode),
                                                  _ptr(out), ctypes.byref(res)))
        finally:
            if cur != prev:
                self.set_stream(prev)
        return out, res.as_dict()

    def torch_device(self):
        import torch
        return torch.device('cuda', self.device)

    def channel_mean(self, inp4, channel, out=None, shape4=None, dtype=None):
        """Multi-channel input (block_components.py:150-159, threshold.py:139-148): the mean of
        the listed channels of a (C, Z, Y, X) volume as the float32 (Z, Y, X) CUDA tensor the
        reference normalizes (np.mean(axis=0) accumulation: float32 for float32 input, float64
        otherwise).  `inp4` is a contiguous CUDA tensor, a CUDA byte tensor holding the raw
        (C, Z, Y, X) data of numpy dtype `dtype` and shape `shape4` (unsigned dtypes need no torch
        support), or a numpy array (uploaded as raw bytes); `channel` is an int or a list of ints
        (order and repeats kept)."""
        import torch
        if shape4 is not None:
            assert hasattr(inp4, 'data_ptr') and inp4.is_cuda and inp4.is_contiguous()
            dt, shape, dev, buf = np.dtype(dtype).name, tuple(int(v) for v in shape4), inp4.device, inp4
            assert len(shape) == 4 and inp4.numel() * inp4.element_size() == int(np.prod(shape)) * np.dtype(dtype).itemsize
        elif hasattr(inp4, 'data_ptr'):
            assert inp4.is_cuda and inp4.is_contiguous() and inp4.dim() == 4
            dt, shape, dev, buf = str(inp4.dtype).replace('torch.', ''), tuple(inp4.shape), inp4.device, inp4
        else:
            a = np.ascontiguousarray(inp4)
            assert a.ndim == 4
            dt, shape, dev = a.dtype.name, a.shape, torch.device('cuda', self.device)
            buf = torch.from_numpy(a.reshape(-1).view(np.uint8)).to(dev)
        if dt not in DTYPES:
            raise TypeError('channel_mean: unsupported dtype %s' % dt)
        chans = _i64([channel] if isinstance(channel, (int, np.integer)) else list(channel))
        if out is None:
            out = torch.empty(shape[1:], dtype=torch.float32, device=dev)
        assert out.dtype == torch.float32 and tuple(out.shape) == tuple(shape[1:]) and out.is_contiguous()
        shape_a = _i64(shape)                         # alive across the call
        _check(load().cc_channel_mean(self._h, _ptr(buf), DTYPES[dt], _ptr(shape_a), _ptr(chans),
                                      len(chans), _ptr(out)))
        return out

    def resize_mask(self, mask, shape, z0=0, nz=None):
        """A mask of another shape than the volume (volume_utils.py:174-184, elf ResizedVolume
        order 0): rows z0 .. z0 + nz of it resized to `shape` by nearest neighbour on the device
        (cc_resize_mask_nearest), as a uint8 CUDA tensor of (nz, Y, X).  `mask` is a numpy array
        or a CUDA uint8 tensor of any (mZ, mY, mX)."""
        import torch
        shape = tuple(int(s) for s in shape)
        nz = shape[0] - z0 if nz is None else int(nz)
        dev = torch.device('cuda', self.device)
        if not hasattr(mask, 'data_ptr'):
            m = np.ascontiguousarray(mask)
            if m.dtype != np.uint8:
                m = (m != 0).astype(np.uint8)
            mask = torch.from_numpy(m).to(dev)
        assert mask.is_cuda and mask.dtype == torch.uint8 and mask.dim() == 3 and mask.is_contiguous()
        out = torch.empty((nz,) + shape[1:], dtype=torch.uint8, device=mask.device)
        torch.cuda.current_stream(mask.device).synchronize()
        ms, vs = _i64(mask.shape), _i64(shape)        # alive across the call
        _check(load().cc_resize_mask_nearest(self._h, _ptr(mask), _ptr(ms), _ptr(vs), int(z0), int(nz), _ptr(out)))
        return out

    def gaussian_smooth_blocks(self, inp, block_shape, sigma, out=None):
        """sigma_prefilter (block_components.py:160-163): per block normalize + Gaussian smoothing
        (vigra.filters.gaussianSmoothing restated, reflected block borders) of a float32 CUDA
        volume; the labelling / threshold calls apply the second normalize.  out may be inp."""
        import torch
        assert hasattr(inp, 'data_ptr') and inp.is_cuda and inp.dtype == torch.float32 and inp.is_contiguous()
        shape, bs = _i64(inp.shape), _i64(block_shape)
        assert len(shape) == 3 and len(bs) == 3
        if out is None:
            out = torch.empty_like(inp)
        assert out.dtype == torch.float32 and out.shape == inp.shape and out.is_contiguous()
        _check(load().cc_gaussian_smooth_blocks(self._h, _ptr(inp), _ptr(shape), _ptr(bs), float(sigma), _ptr(out)))
        return out

    def threshold(self, inp, block_shape, threshold, mode='greater', out=None):
        """Threshold task (threshold.py:131-171): per-block normalize + compare -> uint8.
        `inp` is a float32 torch CUDA tensor; returns a uint8 tensor of the same shape."""
        import torch
        assert hasattr(inp, 'data_ptr') and inp.is_cuda and inp.dtype == torch.float32 and inp.is_contiguous()
        shape = _i64(inp.shape)
        bs = _i64(block_shape)
        assert len(shape) == 3 and len(bs) == 3
        if out is None:
            out = torch.empty(tuple(inp.shape), dtype=torch.uint8, device=inp.device)
        assert out.dtype == torch.uint8 and out.shape == inp.shape and out.is_contiguous()
        _check(load().cc_threshold(self._h, _ptr(inp), _ptr(shape), _ptr(bs), float(threshold),
                                   mode_id(mode), _ptr(out)))
        return out

    AGG = {'mean': 0, 'max': 1, 'min': 2}

    def normalize_channels(self, inp, block_shape, agg='mean', out=None):
        """4-D watershed input (_read_data, watershed_from_seeds.py:127-139) on device: inp =
        the selected channels (C, Z, Y, X) float32 CUDA tensor; per block the 4-D block is
        normalized as one array, then np.mean / np.max / np.min over the channels.  Returns the
        (Z, Y, X) float32 tensor (the watershed input with prenormalized=True)."""
        import torch
        assert inp.is_cuda and inp.dtype == torch.float32 and inp.is_contiguous() and inp.dim() == 4
        shape, bs = _i64(inp.shape[1:]), _i64(block_shape)
        if out is None:
            out = torch.empty(tuple(inp.shape[1:]), dtype=torch.float32, device=inp.device)
        _check(load().cc_normalize_channels(self._h, _ptr(inp), int(inp.shape[0]), _ptr(shape), _ptr(bs),
                                            self.AGG[agg], _ptr(out)))
        return out

    def watershed_from_seeds(self, inp, seeds, block_shape, mask=None, out=None, prenormalized=False):
        """WatershedFromSeeds (watershed/watershed_from_seeds.py:143-273) on device: the seeds
        (uint64 ids < 2^32 - 1, torch int64) grow over the per-block normalized float32 input,
        6-connected inside each block; mask (uint8) -> input 1.0 / output 0 outside it.  out may
        be `seeds` (in place).  prenormalized: the input already holds the normalized values
        (normalize_channels; CC_OPT_WS_PRENORMALIZED).  Returns (labels, relaxation rounds).  See
        include/cc_mi355x.h for the definition (the reference's vu.watershed does not exist:
        parity unpinned)."""
        import torch
        assert hasattr(inp, 'data_ptr') and inp.is_cuda and inp.dtype == torch.float32 and inp.is_contiguous()
        assert seeds.is_cuda and seeds.element_size() == 8 and seeds.shape == inp.shape and seeds.is_contiguous()
        if mask is not None:
            assert mask.is_cuda and mask.dtype == torch.uint8 and mask.shape == inp.shape and mask.is_contiguous()
        shape = _i64(inp.shape)
        bs = _i64(block_shape)
        assert len(shape) == 3 and len(bs) == 3
        if out is None:
            out = torch.empty(tuple(inp.shape), dtype=torch.int64, device=inp.device)
        assert out.element_size() == 8 and out.shape == inp.shape and out.is_contiguous()
        rounds = np.zeros(1, dtype=np.int64)
        _check(load().cc_set_option(self._h, 2, int(bool(prenormalized))))
        try:
            _check(load().cc_watershed_from_seeds(self._h, _ptr(inp), _ptr(seeds), _ptr(mask), _ptr(shape), _ptr(bs),
                                                  _ptr(out), _ptr(rounds)))
        finally:
            _check(load().cc_set_option(self._h, 2, 0))
        return out, int(rounds[0])

    def evaluate(self, seg, gt, block_shape, ignore_label=0):
        """EvaluationWorkflow (evaluation/evaluation_workflow.py:46-84) on device: overlaps per
        block (block_node_labels.py:133-166) + measures (measures.py:81-162).  `seg`, `gt` are
        uint64 (torch int64 / uint64) CUDA tensors of one shape; ignore_label None counts every
        gt voxel.  Returns the cc_eval_result fields as a dict.

        The device table packs (seg, gt) into one 64-bit key (seg < 2^31, gt < 2^32 - 1).  Volumes
        with larger (e.g. sparse 64-bit) ids are first relabelled consecutively on the device
        (relabel_consecutive: order-preserving, 0 stays 0, so the per-block `seg.sum() == 0` skip
        and every measure are unchanged); overlaps() maps the ids back."""
        import torch
        for a in (seg, gt):
            assert hasattr(a, 'data_ptr') and a.is_cuda and a.element_size() == 8 and a.is_contiguous()
            assert a.dtype in (torch.int64, torch.uint64)
        assert seg.shape == gt.shape and seg.dim() == 3
        shape, bs = _i64(seg.shape), _i64(block_shape)
        assert len(bs) == 3
        res = CCEvalResult()
        use_ignore = ignore_label is not None
        # the ctx runs on its own stream: seg / gt may still be in flight on torch's
        torch.cuda.current_stream(seg.device).synchronize()

        self._ev_tables = [None, None]
        # ids that fit the packing are the common case: the device reports ids out of range
        # (EV_ERR_SEG / EV_ERR_GT) and only then are the volumes relabelled (no host-side range
        # scan of the volumes: four reductions over C3's 34 GB tensors took ~40 ms per call)
        rc = load().cc_evaluate(self._h, _ptr(seg), _ptr(gt), _ptr(shape), _ptr(bs), int(use_ignore),
                                int(ignore_label) if use_ignore else 0, ctypes.byref(res))
        if rc == 0:
            return res.as_dict()
        if rc != CC_ERR_ID_RANGE:                      # CC_ERR_ID_RANGE: relabel and evaluate again
            _check(rc)

        def too_large(a, limit):
            v = a.view(torch.int64)
            return bool((v < 0).any()) or bool((v >= limit).any())
        if too_large(seg, 2 ** 31):
            seg, self._ev_tables[0] = self.relabel_consecutive(seg)
        if too_large(gt, 2 ** 32 - 1):
            gt, table = self.relabel_consecutive(gt)
            self._ev_tables[1] = table
            if use_ignore:       # the ignore label in the new id space (an unused id if absent)
                k = np.searchsorted(table[:, 0], np.uint64(ignore_label))
                present = k < len(table) and table[k, 0] == np.uint64(ignore_label)
                ignore_label = int(table[k, 1]) if present else int(table[-1, 1]) + 1
        torch.cuda.current_stream(seg.device).synchronize()
        _check(load().cc_evaluate(self._h, _ptr(seg), _ptr(gt), _ptr(shape), _ptr(bs), int(use_ignore),
                                  int(ignore_label) if use_ignore else 0, ctypes.byref(res)))
        return res.as_dict()

    def overlaps(self):
        """Contingency table of the last evaluate(): (seg_ids, gt_ids, counts) uint64, sorted by
        (seg id, gt id), in the caller's id spaces."""
        L = load()
        n = _check(L.cc_get_overlaps(self._h, None, None, None, 0))
        a, b, c = (np.empty(n, dtype=np.uint64) for _ in range(3))
        _check(L.cc_get_overlaps(self._h, _ptr(a), _ptr(b), _ptr(c), n))
        for k, arr in enumerate((a, b)):
            table = getattr(self, '_ev_tables', [None, None])[k]
            if table is not None:                      # back from the relabelled id space
                arr[:] = table[(arr - table[0, 1]).astype(np.int64), 0]
        o = np.lexsort((b, a))
        return a[o], b[o], c[o]

    def relabel_consecutive(self, labels, out=None, cap_hint=1 << 20):
        """RelabelWorkflow (relabel_workflow.py:10-60, find_labeling.py:84-120) on device:
        returns (relabelled tensor, assignments (n, 2) uint64 [old id, new id]).  `labels` is a
        uint64 (torch int64 / uint64) CUDA tensor; out may be `labels` (in place).  cap_hint: the
        expected number of distinct ids (sizes the host table and the device id set; a larger
        count costs a second call)."""
        import torch
        assert hasattr(labels, 'data_ptr') and labels.is_cuda and labels.element_size() == 8
        assert labels.is_contiguous() and labels.dtype in (torch.int64, torch.uint64)
        if out is None:
            out = torch.empty_like(labels)
        assert out.shape == labels.shape and out.is_contiguous() and out.element_size() == 8
        torch.cuda.current_stream(labels.device).synchronize()
        L = load()
        nu, st = np.zeros(1, dtype=np.uint64), np.zeros(1, dtype=np.uint64)
        cap = max(1, int(cap_hint))
        while True:
            # a table larger than cap is reported (n_unique) before out is touched, so in-place
            # calls are safe: the second call has the exact size
            uniq = np.empty(cap, dtype=np.uint64)
            _check(L.cc_relabel_consecutive(self._h, _ptr(labels), _ptr(out), labels.numel(), _ptr(nu), _ptr(st),
                                            _ptr(uniq), cap))
            if int(nu[0]) <= cap:
                break
            cap = int(nu[0])
        n = int(nu[0])
        uniq = uniq[:n]
        table = np.stack([uniq, np.arange(int(st[0]), int(st[0]) + n, dtype=np.uint64)], axis=1)
        return out, table

    def block_values(self, n_blocks):
        a = np.empty(n_blocks, dtype=np.uint64)
        _check(load().cc_get_block_values(self._h, _ptr(a), n_blocks))
        return a

    def offsets(self, n_blocks):
        a = np.empty(n_blocks, dtype=np.uint64)
        _check(load().cc_get_offsets(self._h, _ptr(a), n_blocks))
        return a

    def lut(self, n_labels):
        a = np.empty(n_labels, dtype=np.uint64)
        _check(load().cc_get_lut(self._h, _ptr(a), n_labels))
        return a

    # ---- stage-level ----
    def block_components(self, inp_dev, block_shape, threshold, mode='greater', mask_dev=None, out_dev=None):
        import torch
        shape = _i64(inp_dev.shape)
        bs = _i64(block_shape)
        nb = int(np.prod([-(-s // b) for s, b in zip(shape, bs)]))
        values = np.empty(nb, dtype=np.uint64)
        if out_dev is None:
            out_dev = torch.empty(tuple(inp_dev.shape), dtype=torch.int64, device=inp_dev.device)
        _check(load().cc_block_components(self._h, _ptr(inp_dev), _ptr(mask_dev), _ptr(shape), _ptr(bs),
                                          float(threshold), mode_id(mode), _ptr(out_dev), _ptr(values), nb))
        return out_dev, values

    def block_faces(self, labels_dev, block_shape, offsets, with_block_flags=False):
        """Deduplicated face pairs; with_block_flags: also the per-block 'has an upper-face pair'
        flags (uint8[n_blocks])."""
        shape = _i64(labels_dev.shape)
        bs = _i64(block_shape)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        flags = np.zeros(len(offsets), dtype=np.uint8) if with_block_flags else None
        # one call when the pairs fit the first buffer (the count comes back either way; a larger
        # count is fetched by a second call with the exact capacity)
        cap = 1 << 20
        pairs = np.empty((cap, 2), dtype=np.uint64)
        n = _check(load().cc_block_faces(self._h, _ptr(labels_dev), _ptr(shape), _ptr(bs), _ptr(offsets),
                                         _ptr(pairs), cap, _ptr(flags)))
        if n > cap:
            pairs = np.empty((n, 2), dtype=np.uint64)
            _check(load().cc_block_faces(self._h, _ptr(labels_dev), _ptr(shape), _ptr(bs), _ptr(offsets),
                                         _ptr(pairs), n, None))
        pairs = pairs[:n].copy() if n < cap else pairs
        return (pairs, flags) if with_block_flags else pairs

    def merge_assignments(self, pairs, n_labels):
        pairs = np.ascontiguousarray(pairs, dtype=np.uint64).reshape(-1, 2)
        lut = np.empty(int(n_labels), dtype=np.uint64)
        _check(load().cc_merge_assignments(self._h, _ptr(pairs), len(pairs), int(n_labels), _ptr(lut)))
        return lut

    def write(self, labels_dev, block_shape, offsets, lut):
        shape = _i64(labels_dev.shape)
        bs = _i64(block_shape)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lut = np.ascontiguousarray(lut, dtype=np.uint64)
        _check(load().cc_write(self._h, _ptr(labels_dev), _ptr(shape), _ptr(bs), _ptr(offsets), _ptr(lut),
                               len(lut)))
        return labels_dev

    def generate_boundary_map(self, shape, origin=(0, 0, 0), seed=0x5EED, out_dev=None, device=None, dither=False):
        import torch
        if out_dev is None:
            out_dev = torch.empty(tuple(int(s) for s in shape), dtype=torch.float32,
                                  device=device if device is not None else 'cuda:%d' % self.device)
        shape_a, origin_a = _i64(shape), _i64(origin)   # keep alive across the call
        _check(load().cc_generate_boundary_map(self._h, _ptr(out_dev), _ptr(shape_a), _ptr(origin_a), int(seed),
                                               int(bool(dither))))
        return out_dev

    # ---- z-slab shards (cluster_tools_amd/distributed.py drives these) ----
    def shard_begin(self, x_dev, block_shape, threshold, mode, z_offset, mask_dev=None):
        shape, bs = _i64(x_dev.shape), _i64(block_shape)
        out = np.zeros(1, dtype=np.uint64)
        _check(load().cc_shard_begin(self._h, _ptr(x_dev), _ptr(mask_dev), _ptr(shape), _ptr(bs),
                                     float(threshold), mode_id(mode), int(z_offset), _ptr(out)))
        return int(out[0])

    def shard_assign(self, id_base):
        _check(load().cc_shard_assign(self._h, int(id_base)))

    def shard_planes(self, bottom_dev=None, top_dev=None):
        _check(load().cc_shard_planes(self._h, _ptr(bottom_dev), _ptr(top_dev)))

    def seam_pairs(self, upper_dev, lower_dev, pairs_dev=None):
        n = upper_dev.numel()
        cap = 0 if pairs_dev is None else pairs_dev.shape[0]
        return _check(load().cc_seam_pairs(self._h, _ptr(upper_dev), _ptr(lower_dev), n, _ptr(pairs_dev), cap))

    def shard_top_plane32(self, top32_dev):
        _check(load().cc_shard_top_plane32(self._h, _ptr(top32_dev)))

    def seam_pairs32(self, upper32_dev, upper_id_base, lower_dev, pairs_dev=None):
        n = upper32_dev.numel()
        cap = 0 if pairs_dev is None else pairs_dev.shape[0]
        return _check(load().cc_seam_pairs32(self._h, _ptr(upper32_dev), int(upper_id_base), _ptr(lower_dev), n,
                                             _ptr(pairs_dev), cap))

    def shard_top_cubes32(self, cubes_dev):
        _check(load().cc_shard_top_cubes32(self._h, _ptr(cubes_dev)))

    def seam_pairs_cubes32(self, upper_cubes_dev, upper_id_base, lower_dev, pairs_dev=None):
        Y, X = lower_dev.shape
        cap = 0 if pairs_dev is None else pairs_dev.shape[0]
        return _check(load().cc_seam_pairs_cubes32(self._h, _ptr(upper_cubes_dev), int(upper_id_base),
                                                   _ptr(lower_dev), int(Y), int(X), _ptr(pairs_dev), cap))

    def shard_finish(self, pairs_dev, n_pairs, out_dev):
        res = CCResult()
        _check(load().cc_shard_finish(self._h, _ptr(pairs_dev) if n_pairs else None, int(n_pairs),
                                      _ptr(out_dev), ctypes.byref(res)))
        return res.as_dict()

    # ---- z-slab shards, one-read-back schedule (distributed.py's default) ----
    def shard_dev_ok(self):
        """Whether this context can run the one-read-back shard schedule (cc_shard_dev_ok)."""
        return bool(load().cc_shard_dev_ok(self._h))

    def shard_dev_begin(self, x_dev, block_shape, threshold, mode, z_offset, sum_dev, mask_dev=None):
        """Local stages of the slab; its sum of block values goes to sum_dev (uint64 on the device)."""
        shape, bs = _i64(x_dev.shape), _i64(block_shape)
        _check(load().cc_shard_dev_begin(self._h, _ptr(x_dev), _ptr(mask_dev), _ptr(shape), _ptr(bs),
                                         float(threshold), mode_id(mode), int(z_offset), _ptr(sum_dev)))

    def shard_dev_assign(self, sums_dev, rank, world):
        _check(load().cc_shard_dev_assign(self._h, _ptr(sums_dev), int(rank), int(world)))

    def shard_dev_top_cubes(self, cubes_dev):
        _check(load().cc_shard_dev_top_cubes(self._h, _ptr(cubes_dev)))

    def shard_dev_seam_pairs(self, upper_cubes_dev, sums_dev, rank, hdr_pairs_dev):
        """hdr_pairs_dev: [cap + 1, 2] int64 -- row 0 (count, redo flags), then the pairs."""
        cap = hdr_pairs_dev.shape[0] - 1
        _check(load().cc_shard_dev_seam_pairs(self._h, _ptr(upper_cubes_dev), _ptr(sums_dev), int(rank),
                                              _ptr(hdr_pairs_dev), int(cap)))

    def shard_dev_finish(self, all_dev, world, sums_dev, out_dev):
        """all_dev: [world * (cap + 1), 2] (every slab's pair buffer).  Returns (result, status):
        status = (redo flags, largest pair count of a slab, n_labels, id base)."""
        cap = all_dev.shape[0] // int(world) - 1
        res = CCResult()
        st = np.zeros(4, dtype=np.uint64)
        _check(load().cc_shard_dev_finish(self._h, _ptr(all_dev), int(world), int(cap), _ptr(sums_dev), _ptr(out_dev),
                                          ctypes.byref(res), _ptr(st)))
        return res.as_dict(), tuple(int(v) for v in st)

    def lut_local(self):
        """The LUT of the last run on this ctx: for a shard, its ids id_base .. id_base + sum."""
        n = 1 << 20
        while True:
            a = np.empty(n, dtype=np.uint64)
            r = load().cc_get_lut(self._h, _ptr(a), n)
            if r >= 0:
                return a[:r]
            if n > 1 << 40:
                _check(r)
            n *= 8

    # ---- profiling ----
    def set_profiling(self, on=True):
        """on: False/0 off, True/1 every launch, 2 only the volume-sized kernels (k_spec, k_pass2)."""
        _check(load().cc_set_profiling(self._h, int(on)))

    def set_empty_job_quirk(self, max_jobs):
        """CC_OPT_EMPTY_JOB_QUIRK: reproduce the reference's empty-job branch
        (merge_assignments.py:115-123) for `max_jobs` face jobs; 0 = off."""
        _check(load().cc_set_option(self._h, 1, int(max_jobs)))

    def set_debug(self, flags):
        """Test hook (include/cc_mi355x.h): 1 = global union-find for intra-block seams."""
        _check(load().cc_set_debug(self._h, int(flags)))

    def reset_profile(self):
        _check(load().cc_reset_profile(self._h))

    def profile(self):
        cap = 64
        names = ctypes.create_string_buffer(8192)
        counts = np.zeros(cap, dtype=np.int64)
        ms = np.zeros(cap, dtype=np.float64)
        n = _check(load().cc_get_profile(self._h, names, 8192, _ptr(counts), _ptr(ms), cap))
        keys = names.value.decode().split(',') if n else []
        return {k: {'count': int(counts[i]), 'total_ms': float(ms[i])} for i, k in enumerate(keys)}


def merge_offsets(values):
    """merge_offsets.py:104-120 through the C ABI (host arithmetic: no device call)."""
    values = np.ascontiguousarray(values, dtype=np.uint64)
    offsets = np.empty_like(values)
    empty = np.empty(len(values), dtype=np.uint8)
    n_labels = np.zeros(1, dtype=np.uint64)
    _check(load().cc_merge_offsets(_ptr(values), len(values), _ptr(offsets), _ptr(empty), _ptr(n_labels)))
    return offsets, np.nonzero(empty)[0], int(n_labels[0])


_COMPRESSION = {'raw': 0, 'gzip': 1}


def n5_read(path, shape, chunks, elem_size, compression, begin, end, out, n_threads=8):
    """cc_n5_read: region [begin, end) of an N5 dataset into the C-order host array `out`."""
    if compression not in _COMPRESSION:
        raise NotImplementedError('n5 compression %s' % compression)
    assert out.flags.c_contiguous and out.dtype.itemsize == elem_size
    sh, ch, b, e = (_i64(v) for v in (shape, chunks, begin, end))
    _check_n5(load_n5().cc_n5_read(os.fsencode(path), len(sh), _ptr(sh), _ptr(ch), int(elem_size),
                                   _COMPRESSION[compression], _ptr(b), _ptr(e), _ptr(out), int(n_threads)))
    return out


def n5_write(path, shape, chunks, elem_size, compression, level, begin, end, data, n_threads=8,
             skip_zero_chunks=False):
    """cc_n5_write: the C-order host array `data` into region [begin, end) of an N5 dataset."""
    if compression not in _COMPRESSION:
        raise NotImplementedError('n5 compression %s' % compression)
    data = np.ascontiguousarray(data)
    assert data.dtype.itemsize == elem_size
    sh, ch, b, e = (_i64(v) for v in (shape, chunks, begin, end))
    _check_n5(load_n5().cc_n5_write(os.fsencode(path), len(sh), _ptr(sh), _ptr(ch), int(elem_size),
                                    _COMPRESSION[compression], int(level), _ptr(b), _ptr(e), _ptr(data),
                                    int(n_threads), int(bool(skip_zero_chunks))))
