"""fmx -- Python (ctypes) binding of libfmx.so, the MI355X many-channel FM
demodulator.  Mirrors include/fmx.h one to one; device buffers are plain
integer addresses (e.g. ``torch.Tensor.data_ptr()`` of a CUDA/HIP tensor).

The binding never falls back to a CPU path: if libfmx.so is missing or no GPU
is present, the calls raise.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMX_LIB") or os.path.join(_HERE, "libfmx.so")  # FMX_LIB: A/B builds (diagnostic)

FMX_OK = 0
FMX_AGC_OFF, FMX_AGC_FAST, FMX_AGC_SLOW = 0, 1, 2
FMX_BLEND_SOFT, FMX_BLEND_NORMAL, FMX_BLEND_AGGRESSIVE = 0, 1, 2
FMX_DEEMPH_50US, FMX_DEEMPH_75US, FMX_DEEMPH_OFF = 0, 1, 2
PARAM = dict(bandwidth_hz=1, w0_hz=2, deemphasis=3, dsp_agc=4, blend=5,
             force_mono=6, force_stereo=7, bandwidth_mode=8, deemph_us=9, deviation_hz=10)
K_FRONTEND, K_STEREO, K_AUDIO, K_RDS, K_RS, K_PILOT, K_FRONTEND_GENERIC, K_BITS = 0, 1, 2, 3, 4, 5, 6, 7
KERNEL_NAMES = ["frontend", "stereo", "audio", "rds", "rs", "pilot", "frontend_generic", "bits"]


class Config(C.Structure):
    _fields_ = [(n, C.c_int) for n in (
        "iq_rate", "dsp_rate", "out_rate", "block", "w0_bandwidth_hz",
        "bandwidth_hz", "dsp_agc", "stereo", "blend", "deemphasis",
        "force_mono", "force_stereo", "rds")]


class RdsGroup(C.Structure):
    _fields_ = [("a", C.c_uint16), ("b", C.c_uint16), ("c", C.c_uint16),
                ("d", C.c_uint16), ("errors", C.c_uint8), ("pad", C.c_uint8),
                ("block_index", C.c_uint32)]


class SignalLevel(C.Structure):
    _fields_ = [("level120", C.c_float), ("level120_smoothed", C.c_float), ("dbfs", C.c_double),
                ("compensated_dbfs", C.c_double), ("hard_clip_ratio", C.c_double),
                ("near_clip_ratio", C.c_double)]


class BlockOut(C.Structure):
    _fields_ = [("d_mpx", C.c_void_p), ("mpx_stride", C.c_int),
                ("d_pcm_l", C.c_void_p), ("d_pcm_r", C.c_void_p),
                ("pcm_stride", C.c_int), ("d_pcm_count", C.c_void_p),
                ("d_stereo", C.c_void_p), ("d_pilot_tenths", C.c_void_p),
                ("d_clip_ratio", C.c_void_p), ("d_groups", C.c_void_p),
                ("groups_stride", C.c_int), ("d_group_count", C.c_void_p),
                ("d_signal", C.c_void_p), ("d_stereo_indicator", C.c_void_p)]


class XdrPiState(C.Structure):
    _fields_ = [("pi_buf", C.c_uint16 * 64), ("pi_err", C.c_uint8 * 8), ("fill", C.c_uint8),
                ("pos", C.c_uint8), ("last_state", C.c_uint8), ("pad", C.c_uint8),
                ("last_value", C.c_uint16), ("pad2", C.c_uint16)]


class SynthConfig(C.Structure):
    _fields_ = [("iq_rate", C.c_int), ("kind", C.c_int), ("amplitude", C.c_float),
                ("noise_std", C.c_float), ("seed_base", C.c_uint32),
                ("max_offset_hz", C.c_int), ("rds_level", C.c_float),
                ("n_bits", C.c_int), ("level_spread_db", C.c_float)]


_lib = None
_OPTIONAL = {"fmx_build_info", "fmx_host_stats", "fmx_diag_set", "fmx_diag_rds_ring"}  # absent from older libraries (A/B against past revisions)


def lib():
    """Load libfmx.so (raises OSError when the HIP extension is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"libfmx.so not built: {LIB_PATH} (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, i, sz, fp = C.c_void_p, C.c_int, C.c_size_t, C.POINTER(C.c_float)
    sig = {
        "fmx_build_info": (C.c_char_p, []),
        "fmx_device_count": (i, []),
        "fmx_create": (i, [C.POINTER(Config), i, i, C.POINTER(vp)]),
        "fmx_destroy": (i, [vp]),
        "fmx_last_error": (C.c_char_p, [vp]),
        "fmx_sync": (i, [vp]),
        "fmx_num_channels": (i, [vp]),
        "fmx_reset": (i, [vp, i]),
        "fmx_retune": (i, [vp, i, i]),
        "fmx_set_param": (i, [vp, i, i, i]),
        "fmx_set_signal_params": (i, [vp, i, i, C.c_double, C.c_double, C.c_double, C.c_double]),
        "fmx_process_block": (i, [vp, vp, sz, i, C.POINTER(BlockOut)]),
        "fmx_decimate": (i, [vp, vp, sz, i, vp, i]),
        "fmx_decimate_u8": (i, [vp, vp, sz, i, vp, sz]),
        "fmx_demod": (i, [vp, vp, i, i, vp, i, vp, i, vp]),
        "fmx_stereo": (i, [vp, vp, i, i, vp, vp, i, vp, vp]),
        "fmx_afpost": (i, [vp, vp, vp, i, i, vp, vp, i, i, vp]),
        "fmx_rds": (i, [vp, vp, i, i, vp, i, vp]),
        "fmx_malloc": (i, [vp, C.POINTER(vp), sz]),
        "fmx_free": (i, [vp, vp]),
        "fmx_memcpy_h2d": (i, [vp, vp, vp, sz]),
        "fmx_memcpy_d2h": (i, [vp, vp, vp, sz]),
        "fmx_memset": (i, [vp, vp, i, sz]),
        "fmx_timing_enable": (i, [vp, i]),
        "fmx_kernel_times": (i, [vp, C.POINTER(C.c_double), C.POINTER(i), i]),
        "fmx_host_stats": (i, [vp, C.POINTER(C.c_double), i]),
        "fmx_diag_set": (i, [vp, i, i]),
        "fmx_diag_rds_ring": (i, [vp, i, fp]),
        "fmx_synth_rds_bits": (i, [C.POINTER(SynthConfig), C.c_uint32, i, vp, vp]),
        "fmx_synth_host": (i, [C.POINTER(SynthConfig), C.c_uint32, i, C.c_int64, i, vp, vp, sz, i]),
        "fmx_synth_device": (i, [vp, C.POINTER(SynthConfig), C.c_uint32, i, C.c_int64, i, vp, vp, sz]),
        "fmx_design_taps": (i, [C.POINTER(Config), i, fp, i]),
        "fmx_resamp_schedule": (i, [C.c_float, i, C.POINTER(C.c_int), fp, i]),
        "fmx_xdr_pi_reset": (None, [C.POINTER(XdrPiState)]),
        "fmx_xdr_rds_lines": (i, [C.POINTER(XdrPiState), vp, i, C.c_char_p, i]),
        "fmx_xdr_scan_line": (i, [vp, vp, vp, i, C.c_char_p, i]),
        "fmx_wav_header": (i, [C.c_uint32, vp]),
        "fmx_pcm_to_s16": (i, [vp, vp, i, i, C.POINTER(C.c_float), vp]),
        "fmx_iq_capture": (i, [C.c_char_p, vp, i, i]),
        "fmx_iq_replay": (i, [C.c_char_p, C.c_longlong, i, vp]),
    }
    for name, (res, args) in sig.items():
        if name in _OPTIONAL and not hasattr(L, name):
            continue  # an older library (A/B runs against a past revision)
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def build_info():
    """fmx_build_info(): "src=<sources' SHA-256, 16 hex> defs=<variant defines>"."""
    L = lib()
    return L.fmx_build_info().decode() if hasattr(L, "fmx_build_info") else "n/a (library without fmx_build_info)"


def make_config(iq_rate=2_400_000, dsp_rate=240_000, out_rate=32_000, block=4096,
                w0_bandwidth_hz=194_000, bandwidth_hz=0, dsp_agc=0, stereo=1,
                blend=1, deemphasis=0, force_mono=0, force_stereo=0, rds=1):
    return Config(iq_rate, dsp_rate, out_rate, block, w0_bandwidth_hz, bandwidth_hz,
                  dsp_agc, stereo, blend, deemphasis, force_mono, force_stereo, rds)


def make_synth(iq_rate=2_400_000, kind=2, amplitude=0.8, noise_std=0.0,
               seed_base=0xF00D, max_offset_hz=5000, rds_level=0.05, n_bits=4096, level_spread_db=0.0):
    return SynthConfig(iq_rate, kind, amplitude, noise_std, seed_base, max_offset_hz,
                       rds_level, n_bits, level_spread_db)


class FmxError(RuntimeError):
    pass


class Handle:
    """One batch of N independent channels on one GPU."""

    def __init__(self, cfg, n_channels, device=0):
        self.L = lib()
        self.cfg = cfg
        self.n = n_channels
        h = C.c_void_p()
        rc = self.L.fmx_create(C.byref(cfg), n_channels, device, C.byref(h))
        self.h = h
        if rc != FMX_OK:
            msg = self.L.fmx_last_error(h).decode() if h.value else "?"
            if h.value:
                self.L.fmx_destroy(h)
            self.h = None
            raise FmxError(f"fmx_create failed ({rc}): {msg}")

    def _ck(self, rc, what):
        if rc != FMX_OK:
            raise FmxError(f"{what} failed ({rc}): {self.L.fmx_last_error(self.h).decode()}")

    def close(self):
        if self.h is not None:
            self.L.fmx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        self._ck(self.L.fmx_sync(self.h), "fmx_sync")

    def reset(self, channel=-1):
        self._ck(self.L.fmx_reset(self.h, channel), "fmx_reset")

    def retune(self, channel=-1, mute_samples=-1):
        """Runtime::reset + retune fade/mute (main.cpp:1028-1042, 1310-1337)."""
        self._ck(self.L.fmx_retune(self.h, channel, mute_samples), "fmx_retune")

    def set_param(self, key, value, channel=-1):
        k = PARAM[key] if isinstance(key, str) else key
        self._ck(self.L.fmx_set_param(self.h, channel, k, value), "fmx_set_param")

    def set_signal_params(self, applied_gain_db=0, gain_comp_factor=0.5, bias_db=-4.0, floor_dbfs=-55.0,
                          ceil_dbfs=-19.0, channel=-1):
        self._ck(self.L.fmx_set_signal_params(self.h, channel, applied_gain_db, gain_comp_factor, bias_db,
                                              floor_dbfs, ceil_dbfs), "fmx_set_signal_params")

    def process_block(self, d_iq, iq_stride, n, out):
        self._ck(self.L.fmx_process_block(self.h, C.c_void_p(d_iq), iq_stride, n, C.byref(out)),
                 "fmx_process_block")

    def decimate(self, d_iq, iq_stride, n_out, d_out, out_stride):
        self._ck(self.L.fmx_decimate(self.h, C.c_void_p(d_iq), iq_stride, n_out,
                                     C.c_void_p(d_out), out_stride), "fmx_decimate")

    def decimate_u8(self, d_iq, iq_stride, n_out, d_out, out_stride):
        self._ck(self.L.fmx_decimate_u8(self.h, C.c_void_p(d_iq), iq_stride, n_out,
                                        C.c_void_p(d_out), out_stride), "fmx_decimate_u8")

    def demod(self, d_iq, in_stride, n, d_mpx, mpx_stride, d_mono=None, mono_stride=0, d_count=None):
        self._ck(self.L.fmx_demod(self.h, C.c_void_p(d_iq), in_stride, n, C.c_void_p(d_mpx), mpx_stride,
                                  C.c_void_p(d_mono), mono_stride, C.c_void_p(d_count)), "fmx_demod")

    def stereo(self, d_mpx, mpx_stride, n, d_l, d_r, lr_stride, d_st=None, d_pilot=None):
        self._ck(self.L.fmx_stereo(self.h, C.c_void_p(d_mpx), mpx_stride, n, C.c_void_p(d_l),
                                   C.c_void_p(d_r), lr_stride, C.c_void_p(d_st), C.c_void_p(d_pilot)),
                 "fmx_stereo")

    def afpost(self, d_l, d_r, in_stride, n, d_ol, d_or, out_stride, cap, d_count):
        self._ck(self.L.fmx_afpost(self.h, C.c_void_p(d_l), C.c_void_p(d_r), in_stride, n,
                                   C.c_void_p(d_ol), C.c_void_p(d_or), out_stride, cap,
                                   C.c_void_p(d_count)), "fmx_afpost")

    def rds(self, d_mpx, mpx_stride, n, d_groups, groups_stride, d_count):
        self._ck(self.L.fmx_rds(self.h, C.c_void_p(d_mpx), mpx_stride, n, C.c_void_p(d_groups),
                                groups_stride, C.c_void_p(d_count)), "fmx_rds")

    def synth_device(self, scfg, ch0, n_ch, sample0, n_samples, d_bits, d_out, out_stride):
        self._ck(self.L.fmx_synth_device(self.h, C.byref(scfg), ch0, n_ch, sample0, n_samples,
                                         C.c_void_p(d_bits), C.c_void_p(d_out), out_stride),
                 "fmx_synth_device")

    def timing_enable(self, on=True, every=1):
        """Per-kernel HIP-event timing; every=N times the launches of every N-th step only."""
        self._ck(self.L.fmx_timing_enable(self.h, max(1, int(every)) if on else 0), "fmx_timing_enable")

    def kernel_times(self):
        nk = len(KERNEL_NAMES)
        ms = (C.c_double * nk)()
        cnt = (C.c_int * nk)()
        self._ck(self.L.fmx_kernel_times(self.h, ms, cnt, nk), "fmx_kernel_times")
        return {KERNEL_NAMES[k]: (ms[k], cnt[k]) for k in range(nk)}

    def diag_set(self, what, value):
        """fmx_diag_set: what 1 = k_rds writes the RDS ring every call."""
        self._ck(self.L.fmx_diag_set(self.h, what, value), "fmx_diag_set")

    def diag_rds_ring(self, channel):
        """The channel's 256-sample RDS FIR ring, oldest first, as a [256, 2]
        float32 array (synchronous; refilled from checkpoints first)."""
        import numpy as np
        out = np.zeros((256, 2), np.float32)
        self._ck(self.L.fmx_diag_rds_ring(self.h, channel, out.ctypes.data_as(C.POINTER(C.c_float))),
                 "fmx_diag_rds_ring")
        return out

    def host_stats(self):
        """Host waits on pinned schedule images since the last call: (waits,
        waits that blocked, milliseconds blocked)."""
        v = (C.c_double * 3)()
        self._ck(self.L.fmx_host_stats(self.h, v, 3), "fmx_host_stats")
        return {"image_waits": int(v[0]), "blocked": int(v[1]), "blocked_ms": round(v[2], 4)}


def synth_rds_bits(scfg, ch0, n_ch):
    import numpy as np
    bits = np.zeros((n_ch, scfg.n_bits), dtype=np.uint8)
    ng = scfg.n_bits // 104
    groups = np.zeros((n_ch, ng, 4), dtype=np.uint16)
    rc = lib().fmx_synth_rds_bits(C.byref(scfg), ch0, n_ch, bits.ctypes.data, groups.ctypes.data)
    if rc != FMX_OK:
        raise FmxError("fmx_synth_rds_bits failed")
    return bits, groups


def synth_host(scfg, ch0, n_ch, sample0, n_samples, bits=None, threads=8):
    import numpy as np
    out = np.zeros((n_ch, 2 * n_samples), dtype=np.uint8)
    bp = bits.ctypes.data if bits is not None else None
    rc = lib().fmx_synth_host(C.byref(scfg), ch0, n_ch, sample0, n_samples, bp,
                              out.ctypes.data, out.shape[1], threads)
    if rc != FMX_OK:
        raise FmxError("fmx_synth_host failed")
    return out


def design_taps(cfg, which):
    import numpy as np
    n = lib().fmx_design_taps(C.byref(cfg), which, None, 0)
    if n < 0:
        raise FmxError("fmx_design_taps failed")
    buf = np.zeros(n, dtype=np.float32)
    lib().fmx_design_taps(C.byref(cfg), which,
                          buf.ctypes.data_as(C.POINTER(C.c_float)), n)
    return buf


def resamp_schedule(del_, n_in):
    import numpy as np
    cap = int(n_in / max(del_, 0.5)) + 16
    packed = np.zeros(cap, dtype=np.int32)
    mu = np.zeros(cap, dtype=np.float32)
    k = lib().fmx_resamp_schedule(C.c_float(del_), n_in,
                                  packed.ctypes.data_as(C.POINTER(C.c_int)),
                                  mu.ctypes.data_as(C.POINTER(C.c_float)), cap)
    return packed[:k], mu[:k]


# ---- host-side formats (fmx_host.cpp): XDR RDS / scan lines, WAV, IQ files ----
class XdrRds:
    """Per-channel XDRServer RDS state (PI debounce) turning fmx_rds_group
    records into the server's "P"/"R" lines."""

    def __init__(self):
        self.st = XdrPiState()
        lib().fmx_xdr_pi_reset(C.byref(self.st))

    def lines(self, groups):
        """groups: list of (a, b, c, d, errors) -> list of lines (no newline)."""
        import numpy as np
        n = len(groups)
        arr = (RdsGroup * max(n, 1))()
        for k, (a, b, c, d, e) in enumerate(groups):
            arr[k] = RdsGroup(a, b, c, d, e, 0, 0)
        cap = 32 * max(n, 1) + 1
        buf = C.create_string_buffer(cap)
        rc = lib().fmx_xdr_rds_lines(C.byref(self.st), C.cast(arr, C.c_void_p), n, buf, cap)
        if rc < 0:
            raise FmxError(f"fmx_xdr_rds_lines failed ({rc})")
        return buf.value.decode().splitlines()


def xdr_scan_line(freq_khz, level_sum, reads):
    import numpy as np
    f = np.ascontiguousarray(freq_khz, dtype=np.int32)
    s = np.ascontiguousarray(level_sum, dtype=np.float64)
    r = np.ascontiguousarray(reads, dtype=np.int32)
    cap = 24 * len(f) + 2
    buf = C.create_string_buffer(cap)
    rc = lib().fmx_xdr_scan_line(f.ctypes.data, s.ctypes.data, r.ctypes.data, len(f), buf, cap)
    if rc < 0:
        raise FmxError(f"fmx_xdr_scan_line failed ({rc})")
    return buf.value.decode()


def wav_header(data_bytes):
    import numpy as np
    h = np.zeros(44, dtype=np.uint8)
    lib().fmx_wav_header(data_bytes, h.ctypes.data)
    return h.tobytes()


def pcm_to_s16(left, right, volume_percent=100, volume_scale=0.85):
    """Returns (interleaved int16 array, new volume_scale)."""
    import numpy as np
    l = np.ascontiguousarray(left, dtype=np.float32)
    r = np.ascontiguousarray(right, dtype=np.float32)
    out = np.zeros(2 * len(l), dtype=np.int16)
    vs = C.c_float(volume_scale)
    rc = lib().fmx_pcm_to_s16(l.ctypes.data, r.ctypes.data, len(l), volume_percent, C.byref(vs), out.ctypes.data)
    if rc < 0:
        raise FmxError("fmx_pcm_to_s16 failed")
    return out, vs.value


def iq_capture(path, iq, append=True):
    import numpy as np
    a = np.ascontiguousarray(iq, dtype=np.uint8)
    rc = lib().fmx_iq_capture(path.encode(), a.ctypes.data, a.size // 2, 1 if append else 0)
    if rc < 0:
        raise FmxError("fmx_iq_capture failed")
    return rc


def iq_replay(path, sample_offset, n_samples):
    import numpy as np
    out = np.zeros(2 * n_samples, dtype=np.uint8)
    k = lib().fmx_iq_replay(path.encode(), sample_offset, n_samples, out.ctypes.data)
    if k < 0:
        raise FmxError("fmx_iq_replay failed")
    return out[:2 * k]
