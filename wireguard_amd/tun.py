"""Host-side mirror of the reference's `tun` hot-path interface over the C ABI.

Names, argument meaning and error behaviour follow /root/reference/tun:
  checksum(b, initial)                     tun/checksum.go:152-167
  checksum_valid(pkt, iph_len, proto, v6)  tun/gro.go:554-612
  gso_none_checksum(read_buf, start, off)  tun/gro.go:1497-1517
  gso_split(read_buf, hdr, bufs, sizes, offset, is_v6)      tun/gro.go:1373-1493
  handle_virtio_read(read_buf, bufs, sizes, offset)         tun/tun.go:514-632
  handle_gro(bufs, lens, offset, can_udp_gro)               tun/gro.go:1326-1367
Go's `(n int, err error)` pairs become `(n, err)` tuples where `err` is None
or a WgcsError carrying the status code (ErrTooManySegments keeps its n).

Batch entry points (`checksum_batch`, `gso_split_batch`) take device
pointers (ints) or torch tensors; torch is only used as the HBM allocator.
Every byte is processed by the gfx950 kernels in libwgcsum.so.
"""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np

from . import _lib
from ._lib import (MODE_FOLD, MODE_L4_FILL, MODE_VALIDATE, MODE_PARTIAL, MODE_IP4HDR, F_INPLACE, PKT_V6,
                   VirtioHdr, WgcsError)

# wgcs_pkt (include/wgcsum.h, ABI 2): 48-bit arena offset split in two fields,
# pseudo-header protocol, flags (PKT_V6), length, csum_start, u16 csum_offset
PKT_DTYPE = np.dtype(
    [("off_lo", "<u4"), ("off_hi", "<u2"), ("proto", "u1"), ("flags", "u1"), ("len", "<u4"),
     ("csum_start", "<u2"), ("csum_offset", "<u2")]
)
IPPROTO_TCP, IPPROTO_UDP = 6, 17


def set_pkt_off(pkts: np.ndarray, off) -> None:
    """Store arena offsets (< 2**48) into a PKT_DTYPE array."""
    off = np.asarray(off, dtype=np.uint64)
    pkts["off_lo"] = (off & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    pkts["off_hi"] = (off >> np.uint64(32)).astype(np.uint16)


def pkt_off(pkts: np.ndarray) -> np.ndarray:
    """Arena offsets of a PKT_DTYPE array (uint64)."""
    return pkts["off_lo"].astype(np.uint64) | (pkts["off_hi"].astype(np.uint64) << np.uint64(32))
GSO_JOB_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("flags", "<u4")])  # wgcs_gso_job
GSO_JOB_RAW, GSO_JOB_V6 = 0x1, 0x2  # WGCS_GSO_JOB_*: gsoSplit with the job's own virtio header / isV6


def gso_job_spare(n: int) -> int:
    """WGCS_GSO_JOB_SPARE(n): n bytes of readBuf's spare capacity follow the job in the arena."""
    return min(n, 255) << 8
# wgcs_batch (include/wgcsum.h): one batch of wgcs_checksum_batches
BATCH_DTYPE = np.dtype([("arena", "<u8"), ("pkts", "<u8"), ("initial", "<u8"), ("out", "<u8"), ("n", "<u4"),
                        ("pad", "<u4")])
# wgcs_gro_buf / wgcs_gro_call (include/wgcsum.h): a device-resident Tun.Write batch
GRO_BUF_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("cap", "<u4")])
GRO_CALL_DTYPE = np.dtype([("first", "<u4"), ("n", "<u4"), ("offset", "<i4"), ("flags", "<u4")])
GRO_CAN_UDP = 0x1
GRO_MAX_CALL = 128

VIRTIO_NET_HDR_LEN = 10
VIRTIO_NET_HDR_F_NEEDS_CSUM = 1
VIRTIO_NET_HDR_GSO_NONE = 0
VIRTIO_NET_HDR_GSO_TCPV4 = 1
VIRTIO_NET_HDR_GSO_TCPV6 = 4
VIRTIO_NET_HDR_GSO_UDP_L4 = 5

__all__ = [
    "Device", "Stager", "WriteStager", "PKT_DTYPE", "GSO_JOB_DTYPE", "GRO_BUF_DTYPE", "GRO_CALL_DTYPE",
    "GRO_CAN_UDP", "GRO_MAX_CALL", "MODE_FOLD", "MODE_L4_FILL", "MODE_VALIDATE", "MODE_PARTIAL",
    "MODE_IP4HDR", "F_INPLACE", "PKT_V6", "IPPROTO_TCP", "IPPROTO_UDP", "VirtioHdr", "WgcsError", "set_pkt_off",
    "pkt_off",
]


def _ptr(x) -> int | None:
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):  # torch tensor
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take a pointer of {type(x)}")


def _np_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        assert buf.dtype == np.uint8
        return buf
    return np.frombuffer(buf, dtype=np.uint8)


class Device:
    """One HIP context (stream + staging) on one GPU; `device` is the HIP ordinal."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        rc = self.lib.wgcs_init(device, C.byref(h))
        if rc != 0:
            raise WgcsError(rc, self.lib.wgcs_strerror(rc).decode())
        self.h = h
        self.device = device
        self._stagers = weakref.WeakSet()  # closed before the context (wgcs_destroy refuses live write stagers)

    def close(self) -> None:
        """wgcs_destroy; raises (and keeps the context) when the library
        refuses, e.g. while a stager made through raw lib calls is alive."""
        if self.h:
            for st in list(self._stagers):
                st.close()
            rc = self.lib.wgcs_destroy(self.h)
            if rc != 0:
                raise WgcsError(rc, self.lib.wgcs_last_error(self.h).decode() or self.lib.wgcs_strerror(rc).decode())
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ utils
    def _check(self, rc: int) -> None:
        if rc != 0:
            raise WgcsError(rc, self.lib.wgcs_last_error(self.h).decode() or self.lib.wgcs_strerror(rc).decode())

    def _err(self, rc: int):
        if rc == 0:
            return None
        if rc <= -100:  # HIP / allocation failures are exceptions, never values
            self._check(rc)
        return WgcsError(rc, self.lib.wgcs_last_error(self.h).decode() or self.lib.wgcs_strerror(rc).decode())

    @property
    def num_cu(self) -> int:
        return self.lib.wgcs_num_cu(self.h)

    def sync(self) -> None:
        self._check(self.lib.wgcs_sync(self.h))

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """Pinned, device-mapped host memory (wgcs_host_alloc) as a uint8 array;
        release it with host_free(array)."""
        p = C.c_void_p()
        self._check(self.lib.wgcs_host_alloc(self.h, nbytes, C.byref(p)))
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(nbytes,))

    def host_free(self, arr: np.ndarray) -> None:
        self._check(self.lib.wgcs_host_free(self.h, arr.ctypes.data))

    def stream_wait_flag(self, stream, flag: np.ndarray, value: int = 1) -> None:
        """wgcs_stream_wait_flag: work enqueued on `stream` afterwards waits
        until flag[0] == value (flag: a uint32 view of host_alloc memory);
        the host rings it with `flag[0] = value`."""
        s = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.wgcs_stream_wait_flag(self.h, s, flag.ctypes.data, value))

    # ---------------------------------------------------------- device batch
    def checksum_batch(self, mode: int, arena, pkts, n: int, out, initial=None, inplace: bool = False,
                       stream=None) -> None:
        """Asynchronous device-resident batch (HBM in, HBM out) on `stream`
        (an int hipStream_t, a torch stream, or None for the context stream)."""
        s = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.wgcs_checksum_batch(self.h, mode, F_INPLACE if inplace else 0, _ptr(arena), _ptr(pkts),
                                                 _ptr(initial), n, _ptr(out), s))

    @staticmethod
    def batch_list(batches) -> np.ndarray:
        """wgcs_batch array for checksum_batches from (arena, pkts, n, out[,
        initial]) tuples of device pointers / tensors."""
        a = np.zeros(len(batches), BATCH_DTYPE)
        for k, b in enumerate(batches):
            arena, pkts, n, out = b[:4]
            a[k] = (_ptr(arena), _ptr(pkts), _ptr(b[4]) if len(b) > 4 and b[4] is not None else 0, _ptr(out), n, 0)
        return a

    def checksum_batches(self, mode: int, batches: np.ndarray, streams=(), ev_begin=None, ev_end=None,
                         inplace: bool = False) -> None:
        """Enqueue a series of independent batches with one call
        (wgcs_checksum_batches): batches[k] (a batch_list array) on
        streams[k % len(streams)]; ev_begin / ev_end (torch.cuda.Event or raw
        hipEvent_t) bracket every launch."""
        ss = (C.c_void_p * max(len(streams), 1))(*[getattr(s, "cuda_stream", s) for s in streams])
        evb = getattr(ev_begin, "cuda_event", ev_begin)
        eve = getattr(ev_end, "cuda_event", ev_end)
        if (ev_begin is not None and not evb) or (ev_end is not None and not eve):
            raise ValueError("bracket event has no HIP event yet (torch creates it on its first record)")
        self._check(self.lib.wgcs_checksum_batches(self.h, mode, F_INPLACE if inplace else 0, batches.ctypes.data,
                                                   len(batches), ss, len(streams), evb or None, eve or None))

    def gso_split_batch(self, arena, jobs, n_jobs: int, out, out_stride: int, offset: int, max_segs: int, sizes,
                        count, status, stream=None) -> None:
        s = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.wgcs_gso_split_batch(self.h, _ptr(arena), _ptr(jobs), n_jobs, _ptr(out), out_stride,
                                                  offset, max_segs, _ptr(sizes), _ptr(count), _ptr(status), s))

    def handle_gro_batch(self, arena, bufs, calls, n_calls: int, status, n_write, to_write, stream=None) -> None:
        """Device-resident batch of Tun.Write calls (wgcs_handle_gro_batch):
        handleGRO per call, in place on `arena` and the GRO_BUF_DTYPE slice
        headers `bufs`; per call status / n_write, toWrite in `to_write`."""
        s = getattr(stream, "cuda_stream", stream)
        self._check(self.lib.wgcs_handle_gro_batch(self.h, _ptr(arena), _ptr(bufs), _ptr(calls), n_calls, _ptr(status),
                                                   _ptr(n_write), _ptr(to_write), s))

    # ------------------------------------------------------------ host batch
    def checksum_batch_host(self, mode: int, arena: np.ndarray, pkts: np.ndarray, initial=None,
                            inplace: bool = False) -> np.ndarray:
        assert pkts.dtype == PKT_DTYPE
        n = len(pkts)
        out = np.zeros(n, dtype=np.uint8 if mode == MODE_VALIDATE else np.uint16)
        ini = None
        if initial is not None:
            ini = np.ascontiguousarray(initial, dtype=np.uint64)
        self._check(self.lib.wgcs_checksum_batch_host(self.h, mode, F_INPLACE if inplace else 0, _ptr(arena),
                                                      arena.nbytes, _ptr(pkts), _ptr(ini), n, _ptr(out)))
        return out

    # -------------------------------------------------- reference-shaped API
    def checksum(self, b, initial: int = 0) -> int:
        """checksum(b []byte, initial uint64) uint16 -- tun/checksum.go:152."""
        a = _np_u8(bytes(b) if not isinstance(b, np.ndarray) else b)
        out = C.c_uint16(0)
        self._check(self.lib.wgcs_checksum(self.h, _ptr(a) if len(a) else None, len(a), initial & (2**64 - 1),
                                           C.byref(out)))
        return out.value

    def checksum_valid(self, pkt, iph_len: int, proto: int, is_v6: bool, n: int | None = None) -> bool:
        """checksumValid(pkt, iphLen, proto, isV6) -- tun/gro.go:554.  With n,
        the packet is pkt[:n] and the rest of pkt its spare capacity."""
        a = _np_u8(bytes(pkt) if not isinstance(pkt, np.ndarray) else pkt)
        v = C.c_int(0)
        ln = len(a) if n is None else n
        self._check(self.lib.wgcs_checksum_valid_cap(self.h, _ptr(a), ln, len(a), iph_len, proto, int(is_v6),
                                                     C.byref(v)))
        return bool(v.value)

    def gso_none_checksum(self, read_buf, csum_start: int, csum_offset: int):
        """gsoNoneChecksum(readBuf, csumStart, csumOffset) error -- mutates read_buf."""
        a = _np_u8(read_buf)
        return self._err(self.lib.wgcs_gso_none_checksum(self.h, _ptr(a), len(a), csum_start, csum_offset))

    @staticmethod
    def _bufs(bufs):
        u8p = C.POINTER(C.c_uint8)
        arr = (u8p * len(bufs))()
        for i, b in enumerate(bufs):
            arr[i] = C.cast(b.ctypes.data, u8p)
        lens = (C.c_size_t * len(bufs))(*[len(b) for b in bufs])
        return arr, lens

    def gso_split(self, read_buf, hdr: VirtioHdr, bufs: list, sizes: list, offset: int, is_v6: bool,
                  n_read: int | None = None):
        """gsoSplit(readBuf, hdr, bufs, sizes, offset, isV6) (int, error).
        With n_read, readBuf is read_buf[:n_read] and the rest of read_buf its
        spare capacity (wgcs_gso_split_cap)."""
        a = _np_u8(read_buf)
        arr, lens = self._bufs(bufs)
        csz = (C.c_int * len(bufs))()
        n = C.c_int(0)
        nr = len(a) if n_read is None else n_read
        rc = self.lib.wgcs_gso_split_cap(self.h, _ptr(a), nr, len(a), C.byref(hdr), arr, lens, len(bufs), csz, offset,
                                         int(is_v6), C.byref(n))
        sizes[: len(bufs)] = list(csz)
        return n.value, self._err(rc)

    def handle_virtio_read(self, read_buf, bufs: list, sizes: list, offset: int, n_read: int | None = None):
        """handleVirtioRead(readBuf, bufs, sizes, offset) (int, error) -- tun/tun.go:514.
        With n_read, readBuf is read_buf[:n_read] and the rest of read_buf its
        spare capacity (Tun.Read's tun.readBuf[:n]; wgcs_handle_virtio_read_cap)."""
        a = _np_u8(read_buf)
        arr, lens = self._bufs(bufs)
        csz = (C.c_int * len(bufs))()
        n = C.c_int(0)
        if n_read is None:
            rc = self.lib.wgcs_handle_virtio_read(self.h, _ptr(a), len(a), arr, lens, len(bufs), csz, offset,
                                                  C.byref(n))
        else:
            rc = self.lib.wgcs_handle_virtio_read_cap(self.h, _ptr(a), n_read, len(a), arr, lens, len(bufs), csz,
                                                      offset, C.byref(n))
        sizes[: len(bufs)] = list(csz)
        return n.value, self._err(rc)

    def handle_gro(self, bufs: list, lens: list, offset: int, can_udp_gro: bool):
        """handleGRO over Go-slice style buffers: bufs[i] is a numpy array whose
        length is cap(bufs[i]); lens[i] = len(bufs[i]).  Returns
        (to_write, order, new_lens, err): order[i] = index of the original
        buffer now at position i (prepend swaps, gro.go:696-697)."""
        n = len(bufs)
        u8p = C.POINTER(C.c_uint8)
        arr = (u8p * n)()
        for i, b in enumerate(bufs):
            arr[i] = C.cast(b.ctypes.data, u8p)
        orig = {b.ctypes.data: i for i, b in enumerate(bufs)}
        clens = (C.c_size_t * n)(*lens)
        ccaps = (C.c_size_t * n)(*[len(b) for b in bufs])
        tw = (C.c_int * max(n, 1))()
        ntw = C.c_int(0)
        rc = self.lib.wgcs_handle_gro(self.h, arr, clens, ccaps, n, offset, int(can_udp_gro), tw, C.byref(ntw))
        addrs = C.cast(arr, C.POINTER(C.c_void_p))
        order = [orig[addrs[i]] for i in range(n)]
        return list(tw)[: ntw.value], order, list(clens), self._err(rc)


class Ring:
    """The resident per-call ring (include/wgcsum.h wgcs_ring_*): the per-call
    checksumValid / handleVirtioRead without a kernel launch per call -- a
    resident kernel serves request records posted in coherent pinned memory.
    Same arguments, results and errors as Device.checksum_valid /
    Device.handle_virtio_read.  Request bytes in Device.host_alloc memory are
    read in place (zero-copy); other arrays are copied into the ring's staging."""

    def __init__(self, dev: Device, idle_us: int = 0):
        self.dev, self.lib = dev, dev.lib
        h = C.c_void_p()
        dev._check(self.lib.wgcs_ring_create(dev.h, idle_us, C.byref(h)))
        self.h = h
        dev._stagers.add(self)  # destroyed before the context

    def close(self) -> None:
        if self.h:
            self.lib.wgcs_ring_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        """requests served, kernel launches made, and whether the kernel is resident now"""
        r, l, on = C.c_uint64(0), C.c_uint64(0), C.c_int(0)
        self.dev._check(self.lib.wgcs_ring_info(self.h, C.byref(r), C.byref(l), C.byref(on)))
        return {"requests": r.value, "launches": l.value, "running": bool(on.value)}

    def checksum_valid(self, pkt, iph_len: int, proto: int, is_v6: bool, n: int | None = None) -> bool:
        """checksumValid(pkt, iphLen, proto, isV6) -- tun/gro.go:554 (as Device.checksum_valid)."""
        a = _np_u8(bytes(pkt) if not isinstance(pkt, np.ndarray) else pkt)
        v = C.c_int(0)
        ln = len(a) if n is None else n
        self.dev._check(self.lib.wgcs_ring_checksum_valid_cap(self.h, _ptr(a), ln, len(a), iph_len, proto,
                                                              int(is_v6), C.byref(v)))
        return bool(v.value)

    def handle_virtio_read(self, read_buf, bufs: list, sizes: list, offset: int, n_read: int | None = None):
        """handleVirtioRead(readBuf, bufs, sizes, offset) (int, error) -- tun/tun.go:514
        (as Device.handle_virtio_read)."""
        a = _np_u8(read_buf)
        arr, lens = Device._bufs(bufs)
        csz = (C.c_int * len(bufs))()
        n = C.c_int(0)
        nr = len(a) if n_read is None else n_read
        rc = self.lib.wgcs_ring_handle_virtio_read_cap(self.h, _ptr(a), nr, len(a), arr, lens, len(bufs), csz, offset,
                                                       C.byref(n))
        sizes[: len(bufs)] = list(csz)
        return n.value, self.dev._err(rc)


class Stager:
    """Tun.Read batch staging ring (include/wgcsum.h wgcs_stager_*): many TUN
    reads -> one GSO-split launch with pipelined H2D / kernel / D2H.

    Create it with max_segs = len(bufs) and seg_room = len(bufs[i]) - offset of
    the Read caller's buffers; then copy_out() leaves bufs/sizes exactly as
    handleVirtioRead (tun/tun.go:514-632) would for that read.  Results of a
    batch stay readable until depth-1 more batches have been submitted."""

    def __init__(self, dev: Device, depth: int, max_reads: int, max_bytes: int, max_segs: int, seg_room: int):
        self.dev, self.lib = dev, dev.lib
        h = C.c_void_p()
        dev._check(self.lib.wgcs_stager_create(dev.h, depth, max_reads, max_bytes, max_segs, seg_room, C.byref(h)))
        self.h = h
        dev._stagers.add(self)
        self.max_segs = max_segs

    def close(self) -> None:
        if self.h:
            self.lib.wgcs_stager_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, read_buf) -> int:
        a = _np_u8(read_buf)
        idx = C.c_int(0)
        self.dev._check(self.lib.wgcs_stager_push(self.h, _ptr(a), len(a), C.byref(idx)))
        return idx.value

    def push_many(self, reads: list) -> int:
        """Push several reads with one call; returns the first read index."""
        arrs = [_np_u8(r) for r in reads]
        ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data if len(a) else None for a in arrs])
        ns = (C.c_size_t * len(arrs))(*[len(a) for a in arrs])
        first, pushed = C.c_int(0), C.c_int(0)
        self.dev._check(self.lib.wgcs_stager_push_many(self.h, ptrs, ns, len(arrs), C.byref(first), C.byref(pushed)))
        return first.value

    def reserve(self, max_n: int):
        """(read_idx, writable uint8 view of the pinned staging) for a read(2)."""
        p, idx = C.c_void_p(), C.c_int(0)
        self.dev._check(self.lib.wgcs_stager_reserve(self.h, max_n, C.byref(p), C.byref(idx)))
        view = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(max_n,)) if max_n else \
            np.zeros(0, np.uint8)
        return idx.value, view

    def commit(self, read_idx: int, n: int) -> None:
        self.dev._check(self.lib.wgcs_stager_commit(self.h, read_idx, n))

    def submit(self) -> int:
        b = C.c_uint64(0)
        self.dev._check(self.lib.wgcs_stager_submit(self.h, C.byref(b)))
        return b.value

    def wait(self, batch: int) -> None:
        self.dev._check(self.lib.wgcs_stager_wait(self.h, batch))

    def result(self, batch: int, read_idx: int):
        """(n, err, sizes) of one read, handleVirtioRead's return values."""
        st, n = C.c_int(0), C.c_int(0)
        sz = C.c_void_p()
        self.dev._check(self.lib.wgcs_stager_result(self.h, batch, read_idx, C.byref(st), C.byref(n), C.byref(sz),
                                                    None))
        k = self.max_segs if st.value == _lib.ERR_TOO_MANY_SEGMENTS else max(n.value, 0)
        sizes = list(np.ctypeslib.as_array(C.cast(sz, C.POINTER(C.c_int32)), shape=(self.max_segs,))[:k])
        return n.value, self.dev._err(st.value), sizes

    def copy_out(self, batch: int, read_idx: int, bufs: list, sizes: list, offset: int):
        """Scatter one read's segments into bufs[i][offset:]; returns (n, err)."""
        arr, lens = Device._bufs(bufs)
        csz = (C.c_int * len(bufs))()
        n = C.c_int(0)
        rc = self.lib.wgcs_stager_copy_out(self.h, batch, read_idx, arr, lens, len(bufs), csz, offset, C.byref(n))
        if rc in (_lib.ERR_INVALID_ARG, _lib.ERR_NOT_READY, _lib.ERR_HIP):
            self.dev._check(rc)
        sizes[: len(bufs)] = list(csz)
        return n.value, self.dev._err(rc)


class WriteStager:
    """Tun.Write batch staging ring (include/wgcsum.h wgcs_wstager_*): many
    Write calls -> one device-resident handleGRO launch (one workgroup per
    call), pipelined H2D / kernels / D2H.  push(bufs, lens, offset) stages one Write call (bufs: numpy arrays of
    cap(bufs[i]) bytes holding len lens[i], the packet at [offset:lens[i]]);
    result() returns what Tun.Write would write(2) for it (tun/tun.go:687-698)."""

    def __init__(self, dev: Device, depth: int, max_writes: int, max_pkts: int, max_bytes: int):
        self.dev, self.lib = dev, dev.lib
        h = C.c_void_p()
        dev._check(self.lib.wgcs_wstager_create(dev.h, depth, max_writes, max_pkts, max_bytes, C.byref(h)))
        self.h = h
        dev._stagers.add(self)
        self._n = {}

    def close(self) -> None:
        if self.h:
            self.lib.wgcs_wstager_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, bufs: list, lens: list, offset: int, can_udp_gro: bool = True) -> int:
        n = len(bufs)
        ptrs = (C.c_void_p * max(n, 1))(*[b.ctypes.data for b in bufs])
        cl = (C.c_size_t * max(n, 1))(*lens)
        cc = (C.c_size_t * max(n, 1))(*[len(b) for b in bufs])
        idx = C.c_int(0)
        self.dev._check(self.lib.wgcs_wstager_push(self.h, ptrs, cl, cc, n, offset, int(can_udp_gro), C.byref(idx)))
        return idx.value

    def push_pinned(self, bufs: list, lens: list, offset: int, can_udp_gro: bool = True) -> int:
        """Zero-copy push: bufs are numpy views of Device.host_alloc memory,
        left untouched until this slot's results have been read."""
        n = len(bufs)
        ptrs = (C.c_void_p * max(n, 1))(*[b.ctypes.data for b in bufs])
        cl = (C.c_size_t * max(n, 1))(*lens)
        cc = (C.c_size_t * max(n, 1))(*[len(b) for b in bufs])
        idx = C.c_int(0)
        self.dev._check(self.lib.wgcs_wstager_push_pinned(self.h, ptrs, cl, cc, n, offset, int(can_udp_gro),
                                                          C.byref(idx)))
        return idx.value

    def submit(self) -> int:
        b = C.c_uint64(0)
        self.dev._check(self.lib.wgcs_wstager_submit(self.h, C.byref(b)))
        return b.value

    def wait(self, batch: int) -> None:
        self.dev._check(self.lib.wgcs_wstager_wait(self.h, batch))

    def result(self, batch: int, write_idx: int, n: int):
        """(err, to_write, packets): packets[k] = bytes written for to_write[k]
        (virtio header + packet), err a WgcsError or None."""
        st, nw = C.c_int(0), C.c_int(0)
        m = max(n, 1)
        tw = (C.c_int * m)()
        ps = (C.c_void_p * m)()
        pl = (C.c_size_t * m)()
        self.dev._check(self.lib.wgcs_wstager_result(self.h, batch, write_idx, C.byref(st), C.byref(nw), tw, ps, pl))
        pkts = [C.string_at(ps[k], pl[k]) for k in range(nw.value)]
        return self.dev._err(st.value), list(tw)[: nw.value], pkts
