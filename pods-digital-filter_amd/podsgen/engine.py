"""Device-resident pipeline of the digital-filter + PODFS hot path.

    DFSetup (host, tiny) -> Generator.generate()          RNG + x/y/z filters + Lund + rotation
                         -> run_pod()                     mean, C = A'^T A'/ns (+ RCCL all-reduce),
                                                          eigensolve, temporal + spatial modes
                         -> run_fourier()                 shifted DFT + ranking/count on the GPU

Multi-GPU: one process per GPU.  Each rank owns a contiguous slab of inlet rows
(host.row_slab); its partial correlation is summed with ONE torch.distributed
all_reduce (RCCL over xGMI with the "nccl" backend).  Rank 0 solves the eigenproblem
and broadcasts lambda and T[:, :nm]; every rank then forms its slab of the spatial modes.

Eigensolve: pods_syev (register-resident tridiagonalisation + bisection + twisted
factorisation, all eigenvalues and the nm leading vectors) whenever only the truncated
temporal modes are needed (ns <= 4096, 0 <= nm <= 64); pods_syev2 (two-stage: band
reduction on fp64 MFMA, bulge chasing, bisection, band inverse iteration) for
4096 < ns <= 16384; torch.linalg.eigh (rocSOLVER dsyevd) when the full temporal-mode matrix
is requested (verbose output), beyond 16384, or with PODS_EIGEN=torch.

PyTorch is used for device memory, the stream, torch.distributed and that fallback
eigensolve -- nothing else.
"""
import ctypes
import os
import time
import warnings
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from ._lib import DFParams, check, ptr
from .host import DFSetup, dft_twiddles, num_valid_modes, rank_and_count, row_slab, time_axis  # noqa: F401

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def _require_gpu():
    if torch is None or not torch.cuda.is_available():
        raise RuntimeError("podsgen needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")


def shared_device(device=0, dist=None):
    """Does another rank of this job drive the same GPU (e.g. a gloo run of several ranks on one
    device)?  Their persistent grids must then not run at the same time (pods_set_shared_device).
    Decided from the devices themselves: every rank contributes (host name, PCI domain / bus /
    device id) to one all_gather_object, so ranks pinned to one visible GPU each (per-rank
    HIP_VISIBLE_DEVICES) or spread over nodes are not taken as sharing.  A collective: all ranks
    call it together (run_pod does, before its first persistent launch).  Without an initialised
    process group of more than one rank: False.  PODS_SHARED_DEVICE=0/1 overrides."""
    env = os.environ.get("PODS_SHARED_DEVICE")
    if env in ("0", "1"):
        return env == "1"
    if dist is None or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() < 2:
        return False
    import socket
    p = torch.cuda.get_device_properties(device)
    me = (socket.gethostname(), int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id))
    ids = [None] * dist.get_world_size()
    dist.all_gather_object(ids, me)
    return sum(1 for x in ids if tuple(x) == me) > 1


class Context:
    """One pods_ctx bound to a device and to torch's current stream on it."""

    def __init__(self, device=0):
        _require_gpu()
        self.lib = _lib.load()
        self.device = int(device)
        torch.cuda.set_device(self.device)
        self.stream = torch.cuda.current_stream(self.device)
        h = ctypes.c_void_p()
        check(self.lib.pods_create(ctypes.byref(h), self.device), "pods_create")
        self.h = h
        check(self.lib.pods_set_stream(self.h, ctypes.c_void_p(self.stream.cuda_stream)), "pods_set_stream")
        self.shared = None   # decided by detect_sharing() (the override at once)
        if os.environ.get("PODS_SHARED_DEVICE") in ("0", "1"):
            self.detect_sharing(None)
        self._side = None

    def detect_sharing(self, dist):
        """Once per context, before its first persistent launch in a multi-rank run (collective
        when `dist` is an initialised group: every rank calls it, see shared_device)."""
        if self.shared is None:
            self.shared = shared_device(self.device, dist)
            if self.shared:
                check(self.lib.pods_set_shared_device(self.h, 1), "pods_set_shared_device")
        return self.shared

    def corr_mode(self):
        """pods_corr's product arithmetic: 1 = exact int8 modular products + CRT, 0 = fp64 SYRK."""
        m = ctypes.c_int(-1)
        check(self.lib.pods_get_corr_mode(self.h, ctypes.byref(m)), "pods_get_corr_mode")
        return m.value

    def set_corr_mode(self, mode):
        check(self.lib.pods_set_corr_mode(self.h, int(mode)), "pods_set_corr_mode")

    def side_stream(self):
        """A second stream on the device for work that may overlap the main stream's."""
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def spatial_stream(self):
        """The stream one device's spatial-mode pass goes to when it may overlap the next run's
        generation (pipeline(overlap_spatial=True))."""
        if getattr(self, "_spatial", None) is None:
            self._spatial = torch.cuda.Stream(device=self.device)
        return self._spatial

    def gen_stream(self):
        """The stream the next run's random planes and x pass go to (Generator.prefetch_next)."""
        if getattr(self, "_gen", None) is None:
            self._gen = torch.cuda.Stream(device=self.device)
        return self._gen

    def on_stream(self, stream):
        """Context manager: the pods context and torch's current stream are `stream` inside."""
        ctx = self

        class _S:
            def __enter__(self):
                self.main = torch.cuda.current_stream(ctx.device)
                # bind the pods context first: if that fails, nothing has been entered yet
                check(ctx.lib.pods_set_stream(ctx.h, ctypes.c_void_p(stream.cuda_stream)), "pods_set_stream")
                self.tc = torch.cuda.stream(stream)
                self.tc.__enter__()
                return self

            def __exit__(self, *exc):
                try:
                    check(ctx.lib.pods_set_stream(ctx.h, ctypes.c_void_p(self.main.cuda_stream)), "pods_set_stream")
                finally:
                    self.tc.__exit__(*exc)
                return False
        return _S()

    def close(self):
        if getattr(self, "h", None):
            self.lib.pods_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class DeviceSnapshots:
    """Handle on the device snapshot matrix A_T (ns x 3*P_local, snapshot-major).
    The reference's A is (3P, ns) with rows [u(P); v(P); w(P)] (digitalfilters.py:1397)."""
    ctx: Context
    ns: int
    rowlen: int
    j0: int = 0
    j1: int = 0
    kma: int = 0

    def data_ptr(self):
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        check(self.ctx.lib.pods_df_snapshots(self.ctx.h, ctypes.byref(p), ctypes.byref(n)), "pods_df_snapshots")
        return p.value

    def to_host_T(self):
        """A_T as a host (ns, 3*P_local) array (device layout is K-tiled, see podsgen.h)."""
        rowpad = (self.rowlen + 15) // 16 * 16
        raw = np.empty((rowpad // 16, self.ns, 16), dtype=np.float64)
        check(self.ctx.lib.pods_copy(self.ctx.h, ptr(raw), ctypes.c_void_p(self.data_ptr()),
                                     raw.nbytes, 1), "pods_copy")
        return np.ascontiguousarray(raw.transpose(1, 0, 2).reshape(self.ns, rowpad)[:, :self.rowlen])

    def to_host(self):
        """The reference layout A (3*P_local, ns)."""
        return np.ascontiguousarray(self.to_host_T().T)


class Generator:
    """digitalfilters.py main() step loop (:1403-1477) on one GPU / row slab."""

    def __init__(self, setup: DFSetup, device=0, rank=0, world=1, ctx: Optional[Context] = None, dist=None,
                 exchange=None):
        self.setup = setup
        self.ctx = ctx or Context(device)
        self.rank, self.world = rank, world
        self.dist = dist
        self.j0, self.j1 = row_slab(setup.jma, rank, world)
        bx, by, bz = setup.taps()
        rot = setup.rotation()
        rotate = bool(setup.rotated and not np.array_equal(rot, np.eye(3)))
        self._keep = [np.ascontiguousarray(bx), np.ascontiguousarray(by), np.ascontiguousarray(bz),
                      setup.lund_rows(self.j0, self.j1), np.ascontiguousarray(rot, dtype=np.float64)]
        p = DFParams(jma=setup.jma, kma=setup.kma, ns=setup.ns, nfx=setup.nfx, nfy=setup.nfy,
                     nfz=setup.nfz, j0=self.j0, j1=self.j1, lund_mode=setup.lund_mode(),
                     rotate=int(rotate), seed=int(setup.seed) & 0xffffffff, reserved=0,
                     rng_low=-np.sqrt(3.0), rng_range=np.sqrt(3.0) - (-np.sqrt(3.0)))
        self.params = p
        k = self._keep
        check(self.ctx.lib.pods_df_configure(self.ctx.h, ctypes.byref(p), ptr(k[0]), ptr(k[1]), ptr(k[2]),
                                             ptr(k[3]), ptr(k[4])), "pods_df_configure")
        self.rowlen = 3 * (self.j1 - self.j0) * setup.kma
        # several ranks: no rank twists the whole MT19937 stream -- each owns 1/world of it and
        # the segment-start states travel in one all_to_all per generation (exchange_states);
        # PODS_MT_EXCHANGE=0 makes every rank twist the whole stream instead (A/B)
        if exchange is None:
            exchange = world > 1 and dist is not None and os.environ.get("PODS_MT_EXCHANGE", "1") != "0"
        self._xch = None
        if exchange:
            self.enable_exchange(required=False)

    def enable_exchange(self, required=True):
        """pods_df_set_exchange with every rank's slab; the send / receive buffers are torch
        tensors on this device (pods_df_exchange_bind).  The library has no exchange plan for a
        stream too short for it (planes shorter than one 312-word MT block, or fewer substreams
        than ranks: tiny inlets such as 8 x 8 with nf = 2); with required=False every rank then
        twists the whole stream instead (the r4 path, same bits) -- the decision depends only on
        the job's shape, so all ranks take the same one."""
        lib, h = self.ctx.lib, self.ctx.h
        slabs = [row_slab(self.setup.jma, q, self.world) for q in range(self.world)]
        j0s = np.array([a for a, _ in slabs], dtype=np.int32)
        j1s = np.array([b for _, b in slabs], dtype=np.int32)
        rc = lib.pods_df_set_exchange(h, self.world, self.rank, ptr(j0s), ptr(j1s))
        if rc == _lib.PODS_ERR_UNSUPPORTED and not required:
            return False
        check(rc, "pods_df_set_exchange")
        sb = np.zeros(self.world, dtype=np.int64)
        rb = np.zeros(self.world, dtype=np.int64)
        check(lib.pods_df_exchange_sizes(h, ptr(sb), ptr(rb)), "pods_df_exchange_sizes")
        dev = torch.device("cuda", self.ctx.device)
        self._send = torch.empty(max(int(sb.sum()), 16), dtype=torch.uint8, device=dev)
        self._recv = torch.empty(max(int(rb.sum()), 16), dtype=torch.uint8, device=dev)
        check(lib.pods_df_exchange_bind(h, ptr(self._send), ptr(self._recv)), "pods_df_exchange_bind")
        self._xch = ([int(x) for x in sb], [int(x) for x in rb])
        return True

    _a2a = None   # finisher of an all_to_all issued ahead (prefetch_jump)

    def exchange_states(self, async_op=False):
        """The all_to_all of the segment-start states (2.5 KB per rank and plane; every rank calls
        generate() / prefetch_jump() together).  RCCL moves device buffers, ordered after the
        current stream; with async_op the call returns a finisher that makes the current stream
        wait for it.  gloo (CPU transport, e.g. several ranks on one GPU) goes through host copies:
        with async_op the device-to-host copy of the records is enqueued on the current stream (the
        gen stream, behind them) into pinned memory and everything else is left to the finisher --
        it waits for that copy only, runs the all_to_all and uploads the received states on the
        stream current at that point (generate()'s), so the host never waits for the generation
        the records were enqueued beside."""
        sb, rb = self._xch
        d = self.dist
        n_s, n_r = sum(sb), sum(rb)
        if d.get_backend() == "nccl":
            work = d.all_to_all_single(self._recv[:n_r], self._send[:n_s], output_split_sizes=rb,
                                       input_split_sizes=sb, async_op=async_op)
            return (lambda: work.wait()) if async_op else None
        if not async_op:
            send = self._send[:n_s].cpu()
            recv = torch.empty(n_r, dtype=torch.uint8)
            d.all_to_all_single(recv, send, output_split_sizes=rb, input_split_sizes=sb)
            self._recv[:n_r].copy_(recv, non_blocking=False)
            return None
        if getattr(self, "_host_xch", None) is None or self._host_xch[0].numel() != n_s:
            self._host_xch = (torch.empty(n_s, dtype=torch.uint8, pin_memory=True),
                              torch.empty(n_r, dtype=torch.uint8, pin_memory=True))
        send, recv = self._host_xch
        send.copy_(self._send[:n_s], non_blocking=True)
        copied = torch.cuda.Event()
        copied.record()

        def finish():
            copied.synchronize()
            d.all_to_all_single(recv, send, output_split_sizes=rb, input_split_sizes=sb)
            self._recv[:n_r].copy_(recv, non_blocking=True)
            # the pinned buffers are reused by the next exchange: keep the upload ordered before it
            done = torch.cuda.Event()
            done.record()
            self._host_xch_done = done
        prev = getattr(self, "_host_xch_done", None)
        if prev is not None:   # the previous upload from `recv` finished before it is overwritten
            prev.synchronize()
        return finish

    _ahead = None      # event behind the next run's prefetched parts (prefetch_*)
    _ahead_parts = 0   # which parts: PODS_GEN_JUMP, + PODS_GEN_PLANES

    def generate(self, timer=None):
        """The whole generation on the current stream -- or, after prefetch_jump() (and
        prefetch_planes_beside_solver()), the parts not yet done, behind the event of those
        already enqueued on the gen stream.  timer (one device, no exchange): each part is launched
        on its own under timer("gen_<part>") -- the same kernels in the same order, one HIP-event
        pair per kernel (bench.py --config c2)."""
        if timer is not None and self._xch is None:
            rest = _lib.PODS_GEN_ALL
            if self._ahead is not None:
                torch.cuda.current_stream(self.ctx.device).wait_event(self._ahead)
                rest &= ~self._ahead_parts
                self._ahead, self._ahead_parts = None, 0
            for part, name in ((_lib.PODS_GEN_JUMP, "gen_jump"), (_lib.PODS_GEN_PLANES, "gen_planes"),
                               (_lib.PODS_GEN_XPASS, "gen_xpass"), (_lib.PODS_GEN_YZPASS, "gen_yzpass")):
                if rest & part:
                    with timer(name):
                        check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, part), "pods_df_generate_parts")
            return self.snapshots()
        if self._xch is not None:   # the state exchange: own substreams, all_to_all, own segments
            done = 0
            if self._ahead is not None:
                torch.cuda.current_stream(self.ctx.device).wait_event(self._ahead)
                done = self._ahead_parts
                self._ahead, self._ahead_parts = None, 0
            pre = (_lib.PODS_GEN_JUMP | _lib.PODS_GEN_RECORD) & ~done
            if pre:
                check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, pre), "pods_df_generate_parts")
            if self._a2a is not None:   # issued ahead, beside the previous step's work
                self._a2a()
                self._a2a = None
            else:
                self.exchange_states()
            rest = _lib.PODS_GEN_PLANES | _lib.PODS_GEN_XPASS | _lib.PODS_GEN_YZPASS
            check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, rest), "pods_df_generate_parts")
        elif self._ahead is not None:
            torch.cuda.current_stream(self.ctx.device).wait_event(self._ahead)
            rest = _lib.PODS_GEN_ALL & ~self._ahead_parts
            self._ahead, self._ahead_parts = None, 0
            check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, rest), "pods_df_generate_parts")
        else:
            check(self.ctx.lib.pods_df_generate(self.ctx.h), "pods_df_generate")
        return self.snapshots()

    def _on_gen_stream(self, parts, timer, name, wait_main=True):
        tm = timer or (lambda name: _NullCtx())
        gs = self.ctx.gen_stream()
        if wait_main:
            gs.wait_stream(torch.cuda.current_stream(self.ctx.device))
        with self.ctx.on_stream(gs):
            with tm(name):
                check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, parts), "pods_df_generate_parts")
            ev = torch.cuda.Event()
            ev.record(gs)
        self._ahead = ev
        self._ahead_parts |= parts & (_lib.PODS_GEN_ALL | _lib.PODS_GEN_RECORD)

    def prefetch_jump(self, timer=None):
        """Enqueue the NEXT run's MT19937 jump-ahead on the gen stream, after everything the main
        stream holds so far (call it after this run's generation: the substream states are free
        again).  It runs beside this run's mean and centring: an LDS-bound kernel (3 workgroups
        per CU) beside two HBM-bound ones, which it does not slow (r3: 1.27 ms hidden, centring
        2.19 ms either way).  The next generate() waits for it.
        (The random planes were tried on the gen stream too: beside the centring they doubled
        its time -- both stream 7-13 GB through HBM -- and beside the SYRK they took 10.9 ms
        instead of 2.4 and cost the SYRK 2.7 ms, no net gain; spread over 64-256 workgroups they
        took 46-77 ms, each substream being a latency-bound twist chain.)"""
        # with the state exchange the owned substreams' records too (they need only the seed), and
        # the all_to_all of the records, ordered behind them on the gen stream; after
        # prefetch_jump_early only the records (the jump is already on the gen stream)
        parts = _lib.PODS_GEN_JUMP | (_lib.PODS_GEN_RECORD if self._xch is not None else 0)
        if self._early:
            if self._xch is not None:
                self._on_gen_stream(_lib.PODS_GEN_RECORD, timer, "gen_jump_ahead")
            else:   # one device: the jump is already on the gen stream; mark its end
                ev = torch.cuda.Event()
                ev.record(self.ctx.gen_stream())
                self._ahead = ev
            self._ahead_parts |= _lib.PODS_GEN_JUMP
            self._early = False
        else:
            self._on_gen_stream(parts, timer, "gen_jump_ahead")
        if self._xch is not None and self.dist is not None:
            with torch.cuda.stream(self.ctx.gen_stream()):
                self._a2a = self.exchange_states(async_op=True)

    _early = False   # the next run's jump-ahead enqueued by prefetch_jump_early

    def prefetch_jump_early(self, timer=None):
        """With the state exchange: enqueue the NEXT run's jump-ahead on the gen stream BEFORE this
        run's generation (call it first in the step; the following prefetch_jump then adds only the
        records and the all_to_all).  The jump needs the jump-state buffer only, which this run's
        records (prefetched in the previous step) have consumed, so it runs beside this run's
        planes and x / y-z passes instead of spilling into the correlation: at N = 8 the rank's
        mean and residues (~0.7 ms) are shorter than the jump (~0.8 ms), and its 50 KB-LDS
        workgroups then held CUs the persistent SYRK's one-per-CU grid waited for (corr +0.5 ms,
        profiles/r5/rank_probe_c3_final.log).  Does nothing unless this run's jump and records
        were prefetched (its generation would otherwise run them on the main stream)."""
        # with the exchange: after the records prefetched one step earlier; on one device
        # (JUMP_EARLY_N1): after the planes prefetched one step earlier consumed the jump states
        ready = _lib.PODS_GEN_RECORD if self._xch is not None else _lib.PODS_GEN_PLANES
        if self._early or not (self._ahead_parts & ready) or (self._xch is None and not JUMP_EARLY_N1):
            return
        tm = timer or (lambda name: _NullCtx())
        gs = self.ctx.gen_stream()
        # behind everything the main stream holds (the previous step's persistent spectrum
        # kernels must not find generator workgroups in the way, as join_ahead ensures)
        gs.wait_stream(torch.cuda.current_stream(self.ctx.device))
        with self.ctx.on_stream(gs):
            with tm("gen_jump_early"):
                check(self.ctx.lib.pods_df_generate_parts(self.ctx.h, _lib.PODS_GEN_JUMP), "pods_df_generate_parts")
        self._early = True

    def prefetch_planes_beside_solver(self, timer=None):
        """Enqueue the NEXT run's random planes on the gen stream behind the marker the current
        pods_syev records after tridiagonalisation range 4 (r6; range 2 until then:
        pods_syev_marker, PLANES_AFTER): from range 3 on
        the k_trd workgroups hold at most 204 VGPRs per wave (2 waves per SIMD) and <= 42 KB of
        LDS, so the MT generator (16 VGPRs; LDS padded to 55 KB so at most 2 of its workgroups
        share a CU, PODS_GEN_BESIDE_SOLVER) runs beside them and every later range still finds
        room on every CU whatever the dispatch order.  Measured against a marker after range 3
        / 4 with up to 3 or 6 generator workgroups per CU: the solver grows least this way
        (36.5 -> 36.9 ms against 37.1-37.2).  Called right after pods_syev is enqueued (after
        prefetch_jump); does nothing when no marker was recorded (ns <= 1536)."""
        # (JUMP_WITH_PLANES, the default on one device: the next jump, not prefetched beside this
        # run's mean and residues, goes here, ahead of the planes)
        jump = JUMP_WITH_PLANES and self._ahead_parts == 0
        if (self._ahead_parts != _lib.PODS_GEN_JUMP and not jump) or self._xch is not None:
            return
        gs = self.ctx.gen_stream()
        if self.ctx.lib.pods_stream_wait_marker(self.ctx.h, ctypes.c_void_p(gs.cuda_stream)) != _lib.PODS_OK:
            return
        # (the x pass beside ranges 3-7 as well, capped at 2 workgroups per CU, measured no faster
        # in r3: generation -2.2 ms on the main stream, the solver +2.5 ms)
        self._on_gen_stream((_lib.PODS_GEN_JUMP if jump else 0) | _lib.PODS_GEN_PLANES | _lib.PODS_GEN_BESIDE_SOLVER,
                            timer, "gen_planes_ahead", wait_main=False)
        # and the next run's x pass, behind the solver's eigenvalues (pods_syev_marker_tail) with
        # 2 workgroups per CU: beside the eigenvectors of T (20 workgroups), the back-transformation
        # (64) and this run's modes, which leave most CUs idle -- the next generation on the main
        # stream is then its y/z pass alone (PODS_XPASS_BESIDE, above)
        if XPASS_BESIDE and self.ctx.lib.pods_stream_wait_marker_tail(
                self.ctx.h, ctypes.c_void_p(gs.cuda_stream)) == _lib.PODS_OK:
            self._on_gen_stream(_lib.PODS_GEN_XPASS | (_lib.PODS_GEN_BESIDE_SOLVER if XPASS_CAP else 0), timer,
                                "gen_xpass_ahead", wait_main=False)

    def join_ahead(self):
        """Make the current stream wait for the prefetched jump-ahead (if any): called before the
        persistent eigensolver kernels, which must not find generator workgroups in the way."""
        if self._ahead is not None:
            torch.cuda.current_stream(self.ctx.device).wait_event(self._ahead)

    def snapshots(self):
        return DeviceSnapshots(self.ctx, self.setup.ns, self.rowlen, self.j0, self.j1, self.setup.kma)


def load_snapshots(A, ctx: Optional[Context] = None, device=0):
    """Upload a reference-layout host A (3P, ns) for PODFS.POD(A, ...)."""
    ctx = ctx or Context(device)
    A = np.asarray(A, dtype=np.float64)
    AT = np.ascontiguousarray(A.T)
    check(ctx.lib.pods_set_snapshots(ctx.h, ptr(AT), AT.shape[0], AT.shape[1]), "pods_set_snapshots")
    return DeviceSnapshots(ctx, AT.shape[0], AT.shape[1])


@dataclass
class PODResult:
    energy: Optional[np.ndarray]  # all ns eigenvalues, descending (host); None when a SpectrumQueue has them
    num_valid: Optional[int]
    nm: int
    mean: "torch.Tensor"          # (3P_local,)
    T: Optional["torch.Tensor"]   # (ns, ncols) scaled temporal modes (rank 0; others: T[:, :nm])
    phi: "torch.Tensor"           # (3P_local, nm) spatial modes
    C: Optional["torch.Tensor"] = None
    timings: dict = field(default_factory=dict)
    phi_ready: Optional["torch.cuda.Event"] = None   # set when phi is computed on another stream


def _dist_info(dist):
    if dist is None or not dist.is_available() or not dist.is_initialized():
        return None, 0, 1
    return dist, dist.get_rank(), dist.get_world_size()


def allreduce_correlation(dist, C, ns, pack, unpack):
    """Sum the ranks' partial correlations C_g = A_g^T A_g (row slabs) and divide by ns
    (PODFS.py:1455, np.dot(A.T, A)/ns): ONE all_reduce of the packed lower triangle
    (ns(ns+1)/2 doubles, half of C) over RCCL/xGMI.  pack(C) -> packed copies the triangle
    out; unpack(packed, C) writes packed / ns (IEEE-rounded like numpy's) to both triangles,
    so C stays exactly symmetric.  On the GPU these are the pods_pack_lower /
    pods_unpack_lower kernels (no index tensors, one pass each)."""
    packed = pack(C)
    dist.all_reduce(packed)
    unpack(packed, C)
    return C


def device_triangle_ops(ctx):
    """pack/unpack callables for allreduce_correlation on ctx's device (C-ABI kernels)."""
    lib = ctx.lib

    def pack(C):
        n = C.shape[0]
        packed = torch.empty(n * (n + 1) // 2, dtype=torch.float64, device=C.device)
        check(lib.pods_pack_lower(ctx.h, ptr(C), n, ptr(packed)), "pods_pack_lower")
        return packed

    def unpack(packed, C):
        n = C.shape[0]
        check(lib.pods_unpack_lower(ctx.h, ptr(packed), n, float(n), ptr(C)), "pods_unpack_lower")
    return pack, unpack


SYEV_MAX_N = 4096   # pods_syev's on-chip limit (trd_plan)
SYEV2_MAX_N = 16384  # pods_syev2 (two-stage): 64 panel workgroups x 256 rows
SYEV_MAX_VEC = 64
SPLIT_MIN_N = 1024   # below this the fused solve is cheaper than a 64-vector subspace iteration
# the next run's x pass beside this run's eigensolver tail (see prefetch_planes_beside_solver):
# PODS_XPASS_BESIDE = 4 (default): behind the eigenvalues, 2 workgroups per CU; 0: on the main
# stream in the next generation; A/B values 1 / 2: behind the tridiagonalisation / the
# eigenvalues with the full grid, 3: behind the tridiagonalisation with 2 workgroups per CU
# (C3, profiles/r6/xpass_beside_ab.log: 69.1-69.4 / 69.1-69.3 / 68.8 / 68.6-68.7 / 68.05-68.1 ms
# per step for 0 / 1 / 2 / 3 / 4)
_XPB = os.environ.get("PODS_XPASS_BESIDE", "4")
XPASS_BESIDE = _XPB in ("1", "2", "3", "4")
XPASS_WHERE = 1 if _XPB in ("2", "4") else 0
XPASS_CAP = _XPB in ("3", "4")
# A/B: one device, the next run's jump-ahead beside this run's y/z pass instead of beside its mean
# and residues (Generator.prefetch_jump_early)
JUMP_EARLY_N1 = os.environ.get("PODS_JUMP_EARLY_N1", "0") == "1"
# one device: the next run's jump-ahead beside the late tridiagonalisation ranges, ahead of its
# planes, instead of beside this run's mean and residues (r6: C3 67.10-67.11 -> 66.54-66.55 ms per
# step, the correlation 0.65 ms faster, profiles/r6/jump_with_planes_ab.log);
# PODS_JUMP_WITH_PLANES=0 restores the old place
JUMP_WITH_PLANES = os.environ.get("PODS_JUMP_WITH_PLANES", "1") == "1"
# the speculative Fourier stage waits for T only, so it runs beside the spatial pass (r6; it had
# waited for the spatial pass too and then ran beside the next step's y/z pass): C3 dft 4.9 -> 1.4
# ms, main-stream generation 5.64 -> 5.22 ms, spatial 1.24 -> 1.47 ms, step 67.9-68.2 -> 67.9-68.0
# (profiles/r6/dft_beside_spatial_ab.log); PODS_DFT_EARLY=0 restores the old order
DFT_EARLY = os.environ.get("PODS_DFT_EARLY", "1") == "1"
# the tridiagonalisation range after which the next run's random planes start: 4 (r6; C3
# 67.62-67.66 / 67.27-67.34 / 67.24-67.28 ms per step after range 2 / 3 / 4 with the x pass
# beside the tail, profiles/r6/planes_marker_ab.log); PODS_PLANES_AFTER overrides
PLANES_AFTER = int(os.environ.get("PODS_PLANES_AFTER", "4"))
SPLIT_MAX_VEC = 40   # leading pairs a 64-vector block resolves (nm <= 40; beyond, the fused solve)


EIGEN_METHODS = ("auto", "pods", "pods2", "torch", "split")


def _eigen_method(world=1, method=None):
    """The eigensolver path: `method` when a caller forces one (a fallback), else PODS_EIGEN."""
    method = method or os.environ.get("PODS_EIGEN", "auto")
    if method not in EIGEN_METHODS:
        raise ValueError("PODS_EIGEN must be auto, pods, pods2, torch or split")
    return method


def _subspace_ws(ctx, n):
    from .subspace import Subspace
    ws = getattr(ctx, "_subspace", None)
    if ws is None or ws.n != n:
        ws = ctx._subspace = Subspace(ctx, n, 64)
    return ws


def eigvals_full(ctx, C, ns, slot=0):
    """All ns eigenvalues, descending (device tensor): the eigenvalues-only tridiagonalisation
    (pods_eigvals_*, ns <= 4096) or the two-stage solver with no vectors (pods_syev2)."""
    lib = ctx.lib
    lam = torch.empty(ns, dtype=torch.float64, device=C.device)
    if ns <= SYEV_MAX_N:
        check(lib.pods_eigvals_begin(ctx.h, slot, ptr(C), ns), "pods_eigvals_begin")
        rem = ctypes.c_int(0)
        check(lib.pods_eigvals_advance(ctx.h, slot, 1 << 20, ctypes.byref(rem)), "pods_eigvals_advance")
        check(lib.pods_eigvals_fetch(ctx.h, slot, ptr(lam)), "pods_eigvals_fetch")
        return lam, lambda: check(lib.pods_eigvals_status(ctx.h, slot), "pods_eigvals")
    check(lib.pods_syev2(ctx.h, ptr(C), ns, 0, ptr(lam), None), "pods_syev2")
    return lam, lambda: check(lib.pods_syev2_status(ctx.h), "pods_syev2")


def eigvals_full_checked(ctx, C, ns):
    """eigvals_full on the host (numpy, descending), recomputed with torch.linalg.eigvalsh when
    the persistent kernels aborted their hand-off wait (the fused path's fallback, for the
    spectrum alone)."""
    lam_t, status = eigvals_full(ctx, C, ns)
    try:
        status()
    except RuntimeError as exc:
        warnings.warn("podsgen: %s; full spectrum by torch.linalg.eigvalsh" % exc)
        lam_t = torch.flip(torch.linalg.eigvalsh(C), dims=(0,))
    return lam_t.cpu().numpy()


def _split_converged(th, info, tol):
    """The subspace iteration's result is usable: finite Ritz values and a final residual at or
    below the tolerance it iterated to (a rank-deficient C can collapse the damped interval and
    yield NaN; max_degree can stop it above tol)."""
    res = info.get("residual", np.inf)
    return bool(np.all(np.isfinite(th)) and np.isfinite(res) and res <= tol)


class SpectrumQueue:
    """The full spectrum (POD.eigenvalues.dat and the printed valid-mode count: PODFS.py:1309-1320,
    :1339) of one correlation matrix per step, off the critical path of a multi-step run.

    Nothing in a step consumes eigenvalues past lambda_{nm-1}, so the eigenvalues-only
    tridiagonalisation of step s (pods_eigvals_*, 33 ms at ns = 4096) runs on an owner rank,
    spread over that rank's following steps in units of one 512-column range (the bisection is
    the last unit).  Per-step budgets even out the ranks' extra work: rank 0 already carries
    the leading-pair solve, the DFT and the ranking (LEAD_MS), so with E the cost of one
    spectrum and T = (E + LEAD_MS) / world, rank 0 gets max(0, T - LEAD_MS) and the others
    share the rest equally (rank 0 gets none from world ~8 on at C3).  Step s is owned by the
    rank a smooth weighted round robin over those budgets picks (the same sequence on every
    rank), and each rank runs units while it has time credit: every step adds its budget,
    every unit spends its measured cost (UNIT_MS at ns = 4096).  Ranks other than 0 run up to
    LEAD_MS of their units while rank 0 solves (before the broadcast of its result, which
    waits for them) and the rest after their spatial modes.  drain() runs what
    is left (inside a caller's timed region); results() returns {step: eigenvalues} for the
    steps this rank owned.  4096 < ns <= 16384 (BASELINE configs 4 and 5): the same queue over
    the two-stage solver's units (pods_eigvals_* run pods_syev2 without vectors as 32-panel
    stage-1 groups, 1024-sweep chase ranges and the bisection: 17 units at ns = 8192), so the
    spectrum spreads over ranks 1..N-1 instead of one owner solving a whole step at once."""

    # per-unit time (ms) of k_trd column ranges 0..7 and the bisection at ns = 4096 (r6: 512
    # columns x the per-column times of profiles/r6/trd_trace_range0_split.log; r3's were 7.8, 5.5,
    # 4.6, 4.0, 3.0, 2.9, 2.5, 2.2); used only to even out the per-step load
    UNIT_MS = [5.5, 4.1, 3.5, 3.4, 3.0, 2.65, 2.6, 2.4, 1.6]
    # rank 0's own extra work per step at ns = 4096 (leading pairs 5.0, DFT + ranking ~1 ms)
    LEAD_MS = 6.0

    # measured per-unit times (ms) of the two-stage units (profiles/r4/eigvals_units.jsonl,
    # tools/eigvals_units_probe.py): 204 ms per spectrum at 8192, 626 ms at 16384
    UNIT_MS_TWO = {8192: [19.4, 16.2, 13.4, 11.1, 9.3, 8.1, 6.8, 5.9, 13.9, 13.8, 13.7, 13.6, 13.4, 13.3, 13.2, 12.6, 6.2],
                   16384: [53.1, 47.1, 42.9, 38.1, 34.1, 30.1, 26.4, 22.7, 19.3, 16.4, 13.4, 11.1, 9.2, 7.9, 6.6, 5.7, 14.4, 14.4, 14.3, 14.2, 14.1, 14.1, 14.0, 13.9, 13.8, 13.7, 13.6, 13.5, 13.5, 13.4, 13.3, 12.6, 21.4]}

    @staticmethod
    def two_stage_costs(ns):
        """Modelled per-unit cost (ms) of the two-stage units at ns > 4096 (r2/r3 profiles at
        8192: a stage-1 panel 0.22 ms of panel QR + 0.47 (m/8192)^2 ms of updates; a chase
        sweep group ~27 us behind the previous one plus one sweep's drain; bisection 5.2 ms x
        (ns/8192)^2).  Only evens out the per-step load; correctness does not depend on it."""
        B, PU, CU = 32, 32, 512
        panels = [ns - c0 - B for c0 in range(0, ns - B - 1, B)]
        cost = []
        for u in range(0, len(panels), PU):
            cost.append(sum(0.22 + 0.47 * (m / 8192.0) ** 2 for m in panels[u:u + PU]))
        groups = (ns - 1) // 2
        for q0 in range(0, groups, CU):
            cost.append(0.027 * min(CU, groups - q0) + 0.65 * ns / 8192.0)
        cost.append(5.2 * (ns / 8192.0) ** 2)
        return cost

    def __init__(self, ctx, ns, rank=0, world=1, max_slots=None):
        self.ctx, self.ns, self.rank, self.world = ctx, ns, rank, world
        if ns > SYEV_MAX_N:
            self.cost = list(self.UNIT_MS_TWO.get(ns) or self.two_stage_costs(ns))
        else:
            units = (ns - 1) // 512 + 2
            self.cost = self.UNIT_MS if units == len(self.UNIT_MS) else [1.0] * units
        self.units = len(self.cost)
        E = sum(self.cost)
        lead = self.LEAD_MS * (ns / 4096.0) ** 2
        if ns <= SYEV_MAX_N:
            lead *= sum(self.cost) / sum(self.UNIT_MS)
        self.lead = lead
        if world == 1:
            self.budgets = [E]
        else:
            b0 = max(0.0, (E + lead) / world - lead)
            self.budgets = [b0] + [(E - b0) / (world - 1)] * (world - 1)
        self.owners = [r for r in range(world) if self.budgets[r] > 0.0]
        self.budget = self.budgets[rank]
        self._seq, self._cur = [], [0.0] * world
        self.credit = 0.0
        # slots in flight: each two-stage slot (ns > 4096) owns a workspace of ~1.5 ns^2 doubles
        # (3.2 GB at 16384) and keeps its step's C, so a rank that falls behind holds at most two
        # of them (the oldest is finished before a third begins, _slot); a one-stage slot is small
        self.max_slots = max_slots if max_slots is not None else (2 if ns > SYEV_MAX_N else 16)
        self.pending = []      # [step, slot, next unit, lam tensor, C]
        # step -> [lam tensor, abort words (pinned, captured on the stream when the spectrum
        # finished), event behind that copy, C until the words were read as 0]
        self.finished = {}
        self.step_no = 0

    def _finish(self, step, lam, C, flags_async):
        """Step `step`'s spectrum is enqueued in full: capture its abort words now (the slot or
        the two-stage workspace is reused by the next matrix) behind an event."""
        words = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        flags_async(words)
        ev = torch.cuda.Event()
        ev.record()
        self.finished[step] = [lam, words, ev, C]

    def _settle(self, step, wait):
        """Reads step's abort words once its event has passed (waits for it when `wait`): a
        completed spectrum drops its C; an aborted one (the persistent kernels' workgroups could
        not all be resident: another process on the device) is recomputed from C with
        torch.linalg.eigvalsh."""
        ent = self.finished[step]
        if ent[3] is None:
            return
        if not wait and not ent[2].query():
            return
        ent[2].synchronize()
        if int(ent[1][0]) or int(ent[1][1]):
            warnings.warn("podsgen: spectrum of step %d aborted its hand-off wait; torch.linalg.eigvalsh" % step)
            ent[0] = torch.flip(torch.linalg.eigvalsh(ent[3]), dims=(0,))
        ent[3] = None

    def _reap(self):
        for s in list(self.finished):
            self._settle(s, wait=False)

    def owner(self, step):
        """The rank that solves step `step`'s spectrum: smooth weighted round robin over the
        budgets (deterministic, identical on every rank)."""
        total = sum(self.budgets)
        while len(self._seq) <= step:
            for r in range(self.world):
                self._cur[r] += self.budgets[r]
            pick = max(range(self.world), key=lambda r: (self._cur[r], -r))
            self._cur[pick] -= total
            self._seq.append(pick)
        return self._seq[step]

    def _slot(self):
        """A free slot; when all max_slots are in flight, the oldest spectrum is finished first
        (its remaining units run now, ahead of their credit) and its slot reused."""
        used = {p[1] for p in self.pending}
        for s in range(self.max_slots):
            if s not in used:
                return s
        self._complete_oldest()
        return self._slot()

    def _complete_oldest(self):
        lib = self.ctx.lib
        rem = ctypes.c_int(0)
        p = self.pending[0]
        while True:
            check(lib.pods_eigvals_advance(self.ctx.h, p[1], 1, ctypes.byref(rem)), "pods_eigvals_advance")
            self.credit -= self.cost[min(p[2], len(self.cost) - 1)]
            p[2] += 1
            if rem.value == 0:
                break
        self._retire(p)

    def _retire(self, p):
        lib = self.ctx.lib
        check(lib.pods_eigvals_fetch(self.ctx.h, p[1], ptr(p[3])), "pods_eigvals_fetch")
        slot = p[1]
        self._finish(p[0], p[3], p[4],
                     lambda w, slot=slot: check(lib.pods_eigvals_flags_async(self.ctx.h, slot, ptr(w)),
                                                "pods_eigvals_flags_async"))
        self.pending.remove(p)

    def submit(self, C, timer=None, limit=None):
        """Registers this step's matrix (begins its spectrum when this rank owns the step), adds
        the step's credit and runs units while credit lasts -- at most `limit` ms of them (the
        rest is left to run())."""
        tm = timer or (lambda name: _NullCtx())
        s = self.step_no
        self.step_no += 1
        lib = self.ctx.lib
        with tm("eig_full"):
            self._reap()
            self.credit += self.budget
            if self.owner(s) == self.rank:
                slot = self._slot()
                check(lib.pods_eigvals_begin(self.ctx.h, slot, ptr(C), self.ns), "pods_eigvals_begin")
                lam = torch.empty(self.ns, dtype=torch.float64, device=C.device)
                self.pending.append([s, slot, 1, lam, C])
                self.credit -= self.cost[0]
            self._advance(limit=limit)

    def run(self, timer=None):
        """Runs units while this step's credit lasts (after a submit with a limit)."""
        tm = timer or (lambda name: _NullCtx())
        with tm("eig_full"):
            self._reap()
            self._advance()

    def _advance(self, drain=False, limit=None):
        lib = self.ctx.lib
        rem = ctypes.c_int(0)
        spent = 0.0
        while self.pending and (drain or (self.credit > 0.0 and (limit is None or spent < limit))):
            p = self.pending[0]
            spent += self.cost[min(p[2], len(self.cost) - 1)]
            check(lib.pods_eigvals_advance(self.ctx.h, p[1], 1, ctypes.byref(rem)), "pods_eigvals_advance")
            self.credit -= self.cost[min(p[2], len(self.cost) - 1)]
            p[2] += 1
            if rem.value == 0:
                self._retire(p)
        if not self.pending:
            self.credit = min(self.credit, self.budget)  # no banking of idle time

    def drain(self):
        self._advance(drain=True)
        self.credit = 0.0

    def results(self):
        """{step: eigenvalues (numpy, descending)} of the finished steps this rank owned.  A
        spectrum whose persistent kernels aborted their hand-off wait (their workgroups could
        not all be resident: another process on the device) is recomputed with
        torch.linalg.eigvalsh from the step's C, which the queue keeps until its abort words
        (captured when the spectrum finished, _finish) have been read."""
        out = {}
        for s in sorted(self.finished):
            self._settle(s, wait=True)
            out[s] = self.finished[s][0].cpu().numpy()
        return out


def eigen_modes(ctx: Context, C, ns, nm, tol_CN, full_temporal, tm=None, world=1):
    """Eigensolve + sort + valid-mode count + temporal scaling (PODFS.py:1309-1325):
    (lambda descending (numpy), num_valid, nm_trunc, T (ns x ncols device tensor))."""
    return eigen_solve(ctx, C, ns, nm, tol_CN, full_temporal, tm, world)[:4]


SPLIT_TOL = 3e-14    # leading_eigenpairs' residual target (/ theta_0)


def eigen_solve(ctx: Context, C, ns, nm, tol_CN, full_temporal, tm=None, world=1, defer_full=False,
                method=None):
    """Eigensolve + sort + valid-mode count + temporal scaling (PODFS.py:1309-1325).

    Returns (lambda descending (numpy; None when defer_full), num_valid (None when deferred),
    nm_trunc, T (ns x ncols device tensor, ncols = ns if full_temporal else max(nm_trunc, 1)),
    the eigenvalues of T's columns (numpy, descending) that scale the modes).

    Paths (PODS_EIGEN=auto):
      fused  (one device, ns <= 4096): pods_syev -- the on-chip tridiagonalisation, all
             eigenvalues, the nm leading vectors by twisted factorisation + back-transformation;
      split  (several ranks, or PODS_EIGEN=split): the nm leading pairs by Chebyshev-filtered
             subspace iteration on fp64 MFMA (podsgen.subspace, stage "eigh"), which is all the
             step consumes; the full spectrum is computed apart (stage "eig_full": now, or by a
             SpectrumQueue when defer_full);
      pods2  (4096 < ns <= 16384 on one device): the two-stage pods_syev2.
    method forces a path (the fallbacks pass "torch" or "pods"); None reads PODS_EIGEN.
    The split path checks its result (finite, residual <= SPLIT_TOL) and otherwise solves again
    with the fused pods_syev (ns <= 4096) or torch.linalg.eigh."""
    from .subspace import leading_eigenpairs
    tm = tm or (lambda name: _NullCtx())
    lib, dev = ctx.lib, C.device
    method = _eigen_method(world, method)
    nvec = max(min(nm, ns), 1) if nm >= 0 else ns
    fits = not full_temporal and nvec <= SYEV_MAX_VEC
    split = (fits and nvec <= SPLIT_MAX_VEC and ns >= SPLIT_MIN_N and
             (method == "split" or (method == "auto" and (world > 1 or defer_full))))
    use_pods = not split and method in ("auto", "pods") and fits and ns <= SYEV_MAX_N
    use_pods2 = not split and fits and 3 <= ns <= SYEV2_MAX_N and (method == "pods2" or
                                                                     (method == "auto" and not use_pods))
    if method in ("pods", "pods2") and not (use_pods or use_pods2):
        raise ValueError("PODS_EIGEN=%s needs ns <= %d, nm <= %d and truncated temporal modes"
                         % (method, SYEV_MAX_N if method == "pods" else SYEV2_MAX_N, SYEV_MAX_VEC))
    if split:
        with tm("eigh"):
            try:
                th, X, info = leading_eigenpairs(ctx, C, nvec, m=64, tol=SPLIT_TOL, ws=_subspace_ws(ctx, ns))
                ok = _split_converged(th, info, SPLIT_TOL)
                why = "residual %r" % info.get("residual")
            except (np.linalg.LinAlgError, ValueError, FloatingPointError, ZeroDivisionError) as exc:
                ok, why = False, str(exc)
        if not ok:
            alt = "pods" if (fits and ns <= SYEV_MAX_N) else "torch"
            warnings.warn("podsgen: subspace iteration did not converge (%s); solving with %s" % (why, alt))
            return eigen_solve(ctx, C, ns, nm, tol_CN, full_temporal, tm, world, method=alt)
        nv_top = num_valid_modes(th, ns, tol_CN)   # exact when < nvec, else a lower bound
        nmt = nm if (0 <= nm <= nv_top) else nv_top
        ncols = max(min(nmt, nvec), 1)
        T = torch.empty((ns, ncols), dtype=torch.float64, device=dev)
        v0 = ctypes.c_void_p(X.data_ptr() + (ns - 1) * 8)   # descending columns, see below
        with tm("temporal"):
            check(lib.pods_temporal_modes(ctx.h, v0, X.shape[1], -1, ptr(np.ascontiguousarray(th)),
                                          min(nv_top, ncols), ncols, ptr(T)), "pods_temporal_modes")
        if defer_full:
            return None, None, nmt, T, th
        with tm("eig_full"):
            lam_desc = eigvals_full_checked(ctx, C, ns)
        return lam_desc, num_valid_modes(lam_desc, ns, tol_CN), nmt, T, th
    if use_pods or use_pods2:
        lam_t = torch.empty(ns, dtype=torch.float64, device=dev)
        Y = torch.empty((ns, nvec), dtype=torch.float64, device=dev)
        with tm("eigh"):
            try:
                if use_pods:
                    check(lib.pods_syev(ctx.h, ptr(C), ns, nvec, ptr(lam_t), ptr(Y)), "pods_syev")
                    check(lib.pods_syev_status(ctx.h), "pods_syev")
                else:  # two-stage (band reduction + bulge chasing) beyond the on-chip limit
                    check(lib.pods_syev2(ctx.h, ptr(C), ns, nvec, ptr(lam_t), ptr(Y)), "pods_syev2")
                    check(lib.pods_syev2_status(ctx.h), "pods_syev2")
            except RuntimeError as exc:
                # a persistent solver whose workgroups could not all be resident (another
                # process on the device) refuses to launch or aborts its hand-off wait: solve
                # with rocSOLVER on the same device instead of failing the POD
                warnings.warn("podsgen: %s; falling back to torch.linalg.eigh" % exc)
                use_pods = use_pods2 = False
            else:
                lam_desc = lam_t.cpu().numpy()
    if use_pods or use_pods2:
        nvalid = num_valid_modes(lam_desc, ns, tol_CN)
        nmt = nm if (0 <= nm <= nvalid) else nvalid
        ncols = max(min(nmt, nvec), 1)
        T = torch.empty((ns, ncols), dtype=torch.float64, device=dev)
        # pods_temporal_modes reads eigh's ascending columns: column ns-1-j of a view with
        # column stride -1 starting at Y[:, ns-1] is Y[:, j]
        v0 = ctypes.c_void_p(Y.data_ptr() + (ns - 1) * 8)
        with tm("temporal"):
            check(lib.pods_temporal_modes(ctx.h, v0, nvec, -1, ptr(lam_desc), min(nvalid, ncols), ncols,
                                          ptr(T)), "pods_temporal_modes")
        return lam_desc, nvalid, nmt, T, lam_desc[:ncols]
    with tm("eigh"):
        lam, V = torch.linalg.eigh(C)
        lam_desc = torch.flip(lam, dims=(0,)).cpu().numpy()
    nvalid = num_valid_modes(lam_desc, ns, tol_CN)
    nmt = nm if (0 <= nm <= nvalid) else nvalid
    ncols = ns if full_temporal else max(nmt, 1)
    T = torch.empty((ns, ncols), dtype=torch.float64, device=dev)
    with tm("temporal"):
        check(lib.pods_temporal_modes(ctx.h, ptr(V), V.stride(0), V.stride(1), ptr(lam_desc),
                                      min(nvalid, ncols), ncols, ptr(T)), "pods_temporal_modes")
    return lam_desc, nvalid, nmt, T, lam_desc[:ncols]


def _speculation_applies(ns, nm, full_temporal, world, spectrum):
    """One device, the fused pods_syev path, truncated temporal modes: the temporal and spatial
    modes can be enqueued for nm_trunc = nm before the host has read the spectrum."""
    return (world == 1 and spectrum is None and not full_temporal and 1 <= nm <= SYEV_MAX_VEC and
            nm + 2 <= ns <= SYEV_MAX_N and _eigen_method() in ("auto", "pods"))


def eigen_solve_speculative(ctx: Context, C, ns, nm, tol_CN, tm, beside=None):
    """pods_syev, then the temporal modes from the device eigenvalues for nm_trunc = nm -- the
    truncation PODFS.py:1312-1320 gives whenever lambda_{nm-1} passes the valid-mode test (the
    spectrum is sorted, so that one test decides it) -- without a host round trip between the
    eigensolve and the modes.  Returns (T, lam_t, Y, verify); verify() synchronises on the
    eigensolve and returns (lam_desc, nvalid) -- the caller redoes the modes on the host path
    when nvalid < nm -- or raises RuntimeError when the persistent solver aborted."""
    lib, dev = ctx.lib, C.device
    lam_t = torch.empty(ns, dtype=torch.float64, device=dev)
    Y = torch.empty((ns, nm), dtype=torch.float64, device=dev)
    if beside is not None:   # a marker behind a tridiagonalisation range for beside()
        # after range min(4, last - 1) (ranges of 512 columns; none for ns <= 1536, as before)
        klast = (ns - 1) // 512
        check(lib.pods_syev_marker(ctx.h, min(PLANES_AFTER, klast - 1) if klast > 2 else 2), "pods_syev_marker")
        if XPASS_BESIDE:     # and one behind the whole tridiagonalisation (or its eigenvalues)
            check(lib.pods_syev_marker_tail(ctx.h, XPASS_WHERE), "pods_syev_marker_tail")
    with tm("eigh"):
        check(lib.pods_syev(ctx.h, ptr(C), ns, nm, ptr(lam_t), ptr(Y)), "pods_syev")
    if beside is not None:
        beside()
    # the spectrum and the solver's abort words go to pinned host memory behind the solve; the
    # host waits for that event only, not for the modes enqueued after it
    pin = getattr(ctx, "_spec_pin", None)
    if pin is None or pin[0].numel() != ns:
        pin = ctx._spec_pin = (torch.empty(ns, dtype=torch.float64, pin_memory=True),
                               torch.zeros(2, dtype=torch.int32, pin_memory=True))
    lam_h, flags_h = pin
    lam_h.copy_(lam_t, non_blocking=True)
    check(lib.pods_syev_flags_async(ctx.h, ptr(flags_h)), "pods_syev_flags_async")
    solved = torch.cuda.Event()
    solved.record()
    T = torch.empty((ns, nm), dtype=torch.float64, device=dev)
    v0 = ctypes.c_void_p(Y.data_ptr() + (ns - 1) * 8)   # eigh's ascending columns, see eigen_solve
    with tm("temporal"):
        check(lib.pods_temporal_modes_dev(ctx.h, v0, nm, -1, ptr(lam_t), nm, nm, ptr(T)), "pods_temporal_modes_dev")

    def verify():
        solved.synchronize()
        if int(flags_h[0]) or int(flags_h[1]):
            raise RuntimeError("pods_syev: hand-off wait timed out (aborted)")
        lam_desc = lam_h.numpy().copy()
        return lam_desc, num_valid_modes(lam_desc, ns, tol_CN)
    return T, lam_t, Y, verify


def pod_head(snap: DeviceSnapshots, world=1, timer=None, partial=None):
    """The mean and the (partial, when world > 1 or `partial`: not divided by ns, the all-reduce's
    unpack divides) correlation of run_pod (PODFS.py:1451-1455 after main() :1492-1495), enqueued
    on the current stream: returns (C, mean)."""
    ctx, lib = snap.ctx, snap.ctx.lib
    dev = torch.device("cuda", ctx.device)
    tm = timer or (lambda name: _NullCtx())
    mean = torch.empty(snap.rowlen, dtype=torch.float64, device=dev)
    with tm("mean"):
        check(lib.pods_mean(ctx.h, ptr(mean), 1), "pods_mean")
    if ctx.corr_mode() == 0:   # the fp64 SYRK reads A centred in place (main() :1493-1495); the
        with tm("center"):     # int8 correlation subtracts the mean while forming its residues
            check(lib.pods_center(ctx.h), "pods_center")
    C = torch.empty((snap.ns, snap.ns), dtype=torch.float64, device=dev)
    with tm("corr"):
        check(lib.pods_corr(ctx.h, ptr(C), 0 if (world > 1 if partial is None else partial) else 1), "pods_corr")
    return C, mean


def run_pod(snap: DeviceSnapshots, nm, tol_CN=1.0e-15, dist=None, full_temporal=False,
            keep_C=False, timer=None, on_temporal=None, spectrum=None, before_eigen=None, beside_solve=None,
            spatial_stream=None):
    """PODFS.POD (PODFS.py:1294-1393) with correct_for_cell_volumes='false'.

    spectrum: a SpectrumQueue -- the eigenvalues past the nm leading ones are then computed by
    it (spread over the following steps, energy/num_valid of the result are None); without one
    the whole spectrum is computed in this call.

    on_temporal(T, nm_trunc, ready), if given, is called on rank 0 with `ready` an event recorded
    behind the temporal modes (again, superseding the first call, when one device's truncation
    check redoes the modes): on one rank right after the spatial modes are enqueued (so the
    spatial pass does not wait for the host to launch the Fourier stage), on several ranks
    before the broadcasts.  pipeline() starts the Fourier stage there on a side stream that
    waits for `ready` only, so it runs beside the spatial-mode pass.

    beside_solve(), if given, is called right after one device's pods_syev is enqueued
    (pipeline() starts the next run's random planes there, beside the late tridiagonalisation
    ranges).

    before_eigen(), if given, is called once the correlation is enqueued, before the first
    host synchronisation of the eigensolve (pipeline() finishes the previous step's Fourier
    results there, while the device runs this step's SYRK)."""
    ctx, lib = snap.ctx, snap.ctx.lib
    ns = snap.ns
    dist, rank, world = _dist_info(dist)
    if world > 1:   # every rank is here: decide whether ranks share this GPU (persistent-grid lock)
        ctx.detect_sharing(dist)
    dev = torch.device("cuda", ctx.device)
    tm = timer or (lambda name: _NullCtx())
    C, mean = pod_head(snap, world, timer)
    if world > 1:
        with tm("allreduce"):
            allreduce_correlation(dist, C, ns, *device_triangle_ops(ctx))
    if before_eigen is not None:
        before_eigen()
    if _speculation_applies(ns, nm, full_temporal, world, spectrum):
        # the modes are enqueued straight behind the eigensolve; the host reads the spectrum while
        # the device computes them (no idle gap for a round trip), then checks the truncation
        T, lam_t, Y, verify = eigen_solve_speculative(ctx, C, ns, nm, tol_CN, tm, beside=beside_solve)
        phi = torch.empty((snap.rowlen, nm), dtype=torch.float64, device=dev)
        t_ready = None
        if DFT_EARLY or spatial_stream is not None:   # T is complete here: the Fourier stage (and
            t_ready = torch.cuda.Event()                # with spatial_stream the spatial pass) may start
            t_ready.record()
        phi_ready = None
        if spatial_stream is not None:   # the spatial pass off the main stream (the caller joins it)
            spatial_stream.wait_event(t_ready)
            for x in (T, lam_t, phi):
                x.record_stream(spatial_stream)
            with ctx.on_stream(spatial_stream):
                with tm("spatial"):
                    check(lib.pods_spatial_modes_dev(ctx.h, ptr(T), nm, ptr(lam_t), nm, ptr(phi)),
                          "pods_spatial_modes_dev")
                phi_ready = torch.cuda.Event()
                phi_ready.record(spatial_stream)
        else:
            with tm("spatial"):
                check(lib.pods_spatial_modes_dev(ctx.h, ptr(T), nm, ptr(lam_t), nm, ptr(phi)), "pods_spatial_modes_dev")
        if t_ready is None:
            t_ready = torch.cuda.Event()
            t_ready.record()
        if on_temporal is not None:   # the Fourier stage (redone on a miss)
            on_temporal(T, nm, t_ready)
        try:
            lam_desc, nvalid = verify()
        except RuntimeError as exc:   # the persistent solver aborted: the whole solve again (fallback)
            warnings.warn("podsgen: %s; falling back to torch.linalg.eigh" % exc)
            lam_desc = None
        if lam_desc is not None and nvalid >= nm:
            nmt = nm
        else:   # fewer valid modes than nm (or no spectrum): the host path
            if phi_ready is not None:   # the speculative spatial pass is superseded
                torch.cuda.current_stream(dev).wait_event(phi_ready)
                phi_ready = None
            if lam_desc is not None:
                nmt = nvalid
                ncols = max(nmt, 1)
                T = torch.empty((ns, ncols), dtype=torch.float64, device=dev)
                v0 = ctypes.c_void_p(Y.data_ptr() + (ns - 1) * 8)
                with tm("temporal"):
                    check(lib.pods_temporal_modes(ctx.h, v0, nm, -1, ptr(lam_desc), min(nvalid, ncols), ncols,
                                                  ptr(T)), "pods_temporal_modes")
                lam_modes = lam_desc[:ncols]
            else:
                lam_desc, nvalid, nmt, T, lam_modes = eigen_solve(ctx, C, ns, nm, tol_CN, full_temporal, tm,
                                                                  method="torch")
            phi = torch.empty((snap.rowlen, max(nmt, 1)), dtype=torch.float64, device=dev)
            if nmt > 0:
                with tm("spatial"):
                    check(lib.pods_spatial_modes(ctx.h, ptr(T), T.shape[1],
                                                 ptr(np.ascontiguousarray(lam_modes[:nmt])), nmt, ptr(phi)),
                          "pods_spatial_modes")
            t_ready = torch.cuda.Event()
            t_ready.record()
            if on_temporal is not None:   # supersedes the speculative launch
                on_temporal(T, nmt, t_ready)
        return PODResult(energy=lam_desc, num_valid=nvalid, nm=nmt, mean=mean, T=T, phi=phi[:, :nmt],
                         C=C if keep_C else None, phi_ready=phi_ready)
    return pod_tail(ctx, snap, C, mean, nm, tol_CN, dist, full_temporal, keep_C, timer, on_temporal, spectrum)


def pod_tail(ctx, snap, C, mean, nm, tol_CN, dist, full_temporal=False, keep_C=False, timer=None, on_temporal=None,
             spectrum=None, solve_stream=None, c_ready=None):
    """The part of run_pod after the correlation (PODFS.py:1309-1333) on the multi-rank / split
    path: rank 0's eigensolve (the nm leading pairs when a SpectrumQueue takes the rest), the
    broadcasts of lambda and T[:, :nm], every rank's spatial modes of its row slab, and the
    spectrum units.  solve_stream (rank 0): the eigensolve runs there, after the event c_ready
    (C complete), so a caller can have the next step's generation and correlation already on the
    main stream (ShardedSteps); the main stream waits for the solve only before the broadcasts."""
    dist, rank, world = _dist_info(dist)
    lib = ctx.lib
    ns = snap.ns
    dev = torch.device("cuda", ctx.device)
    tm = timer or (lambda name: _NullCtx())
    meta = torch.zeros(4, dtype=torch.int64, device=dev)
    T = lam_desc = nvalid = None
    defer = spectrum is not None
    if defer and rank != 0:   # this rank's spectrum units run while rank 0 solves (about as long
        spectrum.submit(C, timer, limit=spectrum.lead)   # as that takes: rank 0 waits for them at
                                                         # the broadcast), the rest after Phi
    if rank == 0:
        if solve_stream is not None:
            if c_ready is not None:
                solve_stream.wait_event(c_ready)
            with ctx.on_stream(solve_stream):
                lam_desc, nvalid, nmt, T, lam_modes = eigen_solve(ctx, C, ns, nm, tol_CN, full_temporal, tm, world,
                                                                  defer_full=defer)
                t_ready = torch.cuda.Event()
                t_ready.record()
            torch.cuda.current_stream(dev).wait_event(t_ready)
            T.record_stream(torch.cuda.current_stream(dev))
        else:
            lam_desc, nvalid, nmt, T, lam_modes = eigen_solve(ctx, C, ns, nm, tol_CN, full_temporal, tm, world,
                                                              defer_full=defer)
            t_ready = torch.cuda.Event()
            t_ready.record()
        if world > 1 and on_temporal is not None:   # beside the broadcasts and the spatial pass
            on_temporal(T, nmt, t_ready)
        meta[0] = -1 if nvalid is None else nvalid
        meta[1] = nmt
        meta[2] = 0 if lam_desc is None else 1
    if world > 1:
        dist.broadcast(meta, 0)
        nv, nmt, have_full = int(meta[0]), int(meta[1]), bool(meta[2])
        nvalid = None if nv < 0 else nv
        lm = torch.empty(max(nmt, 1), dtype=torch.float64, device=dev)
        if rank == 0:
            lm.copy_(torch.from_numpy(np.ascontiguousarray(lam_modes[:max(nmt, 1)])).to(dev))
        dist.broadcast(lm, 0)
        lam_modes = lm.cpu().numpy()
        if have_full:   # the drop-in path: every rank gets the spectrum (32 KB at ns = 4096)
            lt = torch.empty(ns, dtype=torch.float64, device=dev)
            if rank == 0:
                lt.copy_(torch.from_numpy(lam_desc).to(dev))
            dist.broadcast(lt, 0)
            lam_desc = lt.cpu().numpy()
        Tn = torch.empty((ns, max(nmt, 1)), dtype=torch.float64, device=dev)
        if rank == 0:
            Tn.copy_(T[:, :max(nmt, 1)])
        dist.broadcast(Tn, 0)
        if rank != 0:
            T = Tn
        Tsel, ldT = Tn, Tn.shape[1]
    else:
        Tsel, ldT = T, T.shape[1]
    phi = torch.empty((snap.rowlen, max(nmt, 1)), dtype=torch.float64, device=dev)
    if nmt > 0:
        with tm("spatial"):
            check(lib.pods_spatial_modes(ctx.h, ptr(Tsel), ldT, ptr(np.ascontiguousarray(lam_modes[:nmt])),
                                         nmt, ptr(phi)), "pods_spatial_modes")
    if world == 1 and on_temporal is not None:   # after the spatial pass is enqueued
        on_temporal(T, nmt, t_ready)
    if defer and rank == 0:  # the full spectrum, spread over the following steps (SpectrumQueue)
        spectrum.submit(C, timer)
    elif defer:
        spectrum.run(timer)
    return PODResult(energy=lam_desc, num_valid=nvalid, nm=nmt, mean=mean, T=T, phi=phi[:, :nmt],
                     C=C if keep_C else None)


@dataclass
class FourierResult:
    c: np.ndarray          # (ns, nm) complex64
    c_ind: np.ndarray      # (nm, ns) int32
    c_count: np.ndarray    # (nm,) int64
    FC: np.ndarray         # (sum c_count, 3) float64
    period: float
    time: np.ndarray


def host_rank_and_count(c, et):
    ns, nm = c.shape
    c_ind = np.zeros((nm, ns), dtype=np.int32)
    c_count = np.zeros(nm, dtype=np.int64)
    rows = []
    for i in range(nm):
        c_ind[i], c_count[i] = rank_and_count(c[:, i], et)
        idx = c_ind[i, :c_count[i]]
        blk = np.empty((len(idx), 3), dtype=np.float64)
        blk[:, 0] = idx - ns // 2
        blk[:, 1] = c[idx, i].real
        blk[:, 2] = c[idx, i].imag
        rows.append(blk)
    FC = np.concatenate(rows) if rows else np.zeros((0, 3))
    return c_ind, c_count, FC


def fc_rows(c, c_ind, c_count):
    """FC rows [n - ns//2, Re c, Im c] (float64), mode-major in rank order (PODFS.py:1627-1639)."""
    ns = c.shape[0]
    idx = np.concatenate([c_ind[i, :int(c_count[i])] for i in range(len(c_count))]) if len(c_count) else \
        np.zeros(0, np.int64)
    modes = np.repeat(np.arange(len(c_count)), c_count.astype(np.int64))
    FC = np.empty((len(idx), 3), dtype=np.float64)
    FC[:, 0] = idx - ns // 2
    vals = c[idx, modes]
    FC[:, 1] = vals.real
    FC[:, 2] = vals.imag
    return FC


RANK_MAX_NS = 16384  # pods_fourier_rank's LDS limit


def ensure_twiddles(ctx: Context, ns, time_, period):
    """Upload the DFT's host twiddle table (podsgen.host.dft_twiddles) once per time axis."""
    key = (int(ns), float(period), time_.tobytes())
    if getattr(ctx, "_dft_key", None) != key:
        W = dft_twiddles(ns, time_, period)
        check(ctx.lib.pods_fourier_twiddles(ctx.h, int(ns), ptr(np.ascontiguousarray(time_)), float(period),
                                            ptr(W)), "pods_fourier_twiddles")
        ctx._dft_key = key


def run_fourier(ctx: Context, T, nm, ns, dt, et, timer=None):
    """fourier_coefficients (PODFS.py:1523-1659): DFT and ranking/count on the GPU
    (pods_fourier + pods_fourier_rank); FC assembled on the host from the ranked indices."""
    return launch_fourier(ctx, T, nm, ns, dt, et, timer)()


def launch_fourier(ctx: Context, T, nm, ns, dt, et, timer=None, side=False, ready=None):
    """Enqueue the DFT and the ranking kernels; returns finish() -> FourierResult.

    side=True runs them on the context's side stream (forked from the current stream, or from
    the event `ready` recorded behind T), concurrently with the caller's work on the current
    stream (the spatial modes: an HBM-bound pass beside this VALU-bound one).  finish() copies on that
    stream and the pods context is bound back to the current stream before returning."""
    tm = timer or (lambda name: _NullCtx())
    time_, period = time_axis(ns, dt)
    dev = torch.device("cuda", ctx.device)
    nm = int(nm)
    if nm == 0:
        res = FourierResult(np.zeros((ns, 0), np.complex64), np.zeros((0, ns), np.int32),
                            np.zeros(0, np.int64), np.zeros((0, 3)), period, time_)
        return lambda: res
    time_ = np.ascontiguousarray(time_, dtype=np.float64)
    ensure_twiddles(ctx, ns, time_, period)
    main = torch.cuda.current_stream(dev)
    stream = main
    if side:
        stream = ctx.side_stream()
        if ready is not None:   # T complete; later work on the main stream is not waited for
            stream.wait_event(ready)
        else:
            stream.wait_stream(main)
        T.record_stream(stream)
    with torch.cuda.stream(stream):
        if side:
            check(ctx.lib.pods_set_stream(ctx.h, ctypes.c_void_p(stream.cuda_stream)), "pods_set_stream")
        try:
            cbuf = torch.empty((ns, nm, 2), dtype=torch.float32, device=dev)
            with tm("dft"):
                check(ctx.lib.pods_fourier(ctx.h, ptr(T), T.stride(0), nm, ns,
                                           ptr(np.ascontiguousarray(time_)), float(period), ptr(cbuf)),
                      "pods_fourier")
            ind = cnt = None
            if ns <= RANK_MAX_NS:
                with tm("rank"):
                    ind = torch.empty((nm, ns), dtype=torch.int32, device=dev)
                    cnt = torch.empty(nm, dtype=torch.int64, device=dev)
                    check(ctx.lib.pods_fourier_rank(ctx.h, ptr(cbuf), nm, ns, float(et), ptr(ind), ptr(cnt)),
                          "pods_fourier_rank")
        finally:
            if side:
                check(ctx.lib.pods_set_stream(ctx.h, ctypes.c_void_p(main.cuda_stream)), "pods_set_stream")

    def finish():
        with torch.cuda.stream(stream):
            c = cbuf.cpu().numpy().view(np.complex64).reshape(ns, nm)
            if ind is not None:
                c_ind = ind.cpu().numpy()
                c_count = cnt.cpu().numpy()
                if np.any(c_count < 0):
                    raise IndexError("energy target not reachable (et = %r > 1?)" % et)
                FC = fc_rows(c, c_ind, c_count)
            else:
                c_ind, c_count, FC = host_rank_and_count(c, et)
        return FourierResult(c=c, c_ind=c_ind, c_count=c_count, FC=FC, period=period, time=time_)
    return finish


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class StageTimer:
    """Per-stage GPU time with HIP events on the pipeline's stream (torch events wrap
    hipEvent_t on the current stream, which is the stream the kernels run on)."""

    def __init__(self, enabled=True):
        self.enabled = enabled
        self.events = []

    def __call__(self, name):
        timer = self

        class _C:
            def __enter__(self):
                if timer.enabled:
                    self.a = torch.cuda.Event(enable_timing=True)
                    self.a.record()
                return self

            def __exit__(self, *exc):
                if timer.enabled:
                    b = torch.cuda.Event(enable_timing=True)
                    b.record()
                    timer.events.append((name, self.a, b))
                return False
        return _C()

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, a, b in self.events:
            out[name] = out.get(name, 0.0) + a.elapsed_time(b)
        return out


class FourierBacklog:
    """Fourier results of a multi-step run finished one step late: the host-side part (copies
    of c, the ranking and the FC rows) of step s runs while the device computes step s+1's
    correlation, instead of leaving the device idle between steps.  results[s] is step s's
    FourierResult (None without modes); flush() finishes what is left."""

    def __init__(self):
        self.pending = []
        self.results = []

    def finish_pending(self):
        while self.pending:
            fin = self.pending.pop(0)
            self.results.append(fin() if fin is not None else None)

    flush = finish_pending


def pipeline(setup: DFSetup, device=0, dist=None, full_temporal=False, timer=None, gen=None, spectrum=None,
             backlog=None, prefetch_next=False, overlap_spatial=False):
    """The whole hot path; returns (Generator, PODResult, FourierResult | None).
    spectrum: a SpectrumQueue for multi-step runs (see run_pod).  backlog: a FourierBacklog --
    this step's Fourier result is then finished during the next step (or by backlog.flush())
    and the returned FourierResult is None.  prefetch_next: a next run follows on this
    generator; its random planes and x pass are enqueued on the gen stream right after this
    run's generation: the MT19937 jump-ahead, beside this run's mean and centring
    (Generator.prefetch_jump).

    overlap_spatial (one device, multi-step runs): consecutive runs alternate between the two
    snapshot banks (pods_select_snapshots) and this run's spatial-mode pass goes to its own stream
    behind the temporal modes, so the next run's generation (into the other bank) starts beside
    it; pod.phi is then complete once pod.phi_ready has passed (the main stream waits for it
    before the bank is generated into again, and at once when no next run follows)."""
    dist_, rank, world = _dist_info(dist)
    tm = timer or (lambda name: _NullCtx())
    gen = gen or Generator(setup, device=device, rank=rank, world=world, dist=dist_)
    overlap = overlap_spatial and world == 1
    if overlap:
        bank = getattr(gen, "_sp_bank", 0)
        gen._sp_bank = bank ^ 1
        check(gen.ctx.lib.pods_select_snapshots(gen.ctx.h, bank), "pods_select_snapshots")
        waits = getattr(gen, "_sp_wait", None)
        if waits is None:
            waits = gen._sp_wait = {}
        ev = waits.pop(bank, None)
        if ev is not None:   # the spatial pass that read this bank two runs ago
            torch.cuda.current_stream(gen.ctx.device).wait_event(ev)
    if prefetch_next and JUMP_EARLY_N1:
        gen.prefetch_jump_early(timer)   # A/B: the next jump beside this generation's y/z pass
    with tm("generate"):
        snap = gen.generate()
    # (with the planes beside the solver -- ns > 1536, one device -- the jump goes there too)
    if prefetch_next and not (JUMP_WITH_PLANES and gen._xch is None and (setup.ns - 1) // 512 > 2):
        gen.prefetch_jump(timer)
    pending = []

    def start_fourier(T, nmt, ready):
        pending.append(launch_fourier(gen.ctx, T, nmt, setup.ns, setup.dt_eff, setup.et, timer=timer,
                                      side=True, ready=ready))
    def before_eigen():
        gen.join_ahead()
        if backlog is not None:
            backlog.finish_pending()
    beside = (lambda: gen.prefetch_planes_beside_solver(timer)) if prefetch_next else None
    pod = run_pod(snap, setup.nm, dist=dist_, full_temporal=full_temporal, timer=timer,
                  on_temporal=start_fourier, spectrum=spectrum, before_eigen=before_eigen, beside_solve=beside,
                  spatial_stream=gen.ctx.spatial_stream() if overlap else None)
    if pod.phi_ready is not None:
        if prefetch_next:
            gen._sp_wait[bank] = pod.phi_ready
        else:
            torch.cuda.current_stream(gen.ctx.device).wait_event(pod.phi_ready)
    # the last launch counts (a speculative Fourier launch is superseded when the truncation
    # check redoes the modes)
    if backlog is not None:
        backlog.pending.append(pending[-1] if pending else None)
        return gen, pod, None
    fo = pending[-1]() if pending else None
    return gen, pod, fo


class ShardedSteps:
    """Several ranks, several steps (bench.py --gpus N > 1): the POD tail of step k-1 runs while
    the device already has step k's generation and correlation.

    step() enqueues step k's generation (into snapshot bank k % 2, pods_select_snapshots) and its
    mean + partial correlation, THEN runs step k-1's tail (pod_tail: rank 0 solves for the nm
    leading pairs on its own stream behind the event of step k-1's all-reduce, so the device runs
    that latency-bound solve beside step k's HBM / MFMA-bound kernels; the other ranks run their
    spectrum units; broadcasts of lambda and T; every rank's spatial modes of step k-1 from bank
    (k-1) % 2; the Fourier stage on rank 0), and then issues step k's all-reduce asynchronously
    (the next step's generation runs beside it; the tail waits for it and unpacks C).  Every result is
    that of the unpipelined order bit for bit (same kernels on the same inputs); pipelined=False
    (PODS_PIPELINE=0) runs each step's tail right after its own all-reduce.  results[k] is step
    k's PODResult once its tail has run; flush() runs the last tail.  collectives=True runs the
    all-reduce through the process group even at world 1 (a one-rank group: a sum of one, exactly
    the divided SYRK's bits), so a single device exercises the backend's collective path (tests)."""

    def __init__(self, setup: DFSetup, gen, dist, spectrum=None, backlog=None, pipelined=None, collectives=None):
        self.setup, self.gen, self.dist = setup, gen, dist
        self.spectrum, self.backlog = spectrum, backlog
        if pipelined is None:
            pipelined = os.environ.get("PODS_PIPELINE", "1") != "0"
        self.pipelined = pipelined
        self.k = 0
        self.pending = None
        self.results = []
        _, self.rank, self.world = _dist_info(dist)
        self._solve = None
        self._spec_done = None
        self.collectives = self.world > 1 if collectives is None else bool(collectives)

    def _solve_stream(self):
        if self._solve is None:
            self._solve = torch.cuda.Stream(device=self.gen.ctx.device)
        return self._solve

    def step(self, timer=None, prefetch_next=False, seed=None):
        """One step; seed: a new np.random.seed for this step's field (pods_df_set_seed; must not
        be combined with a jump-ahead prefetched under the previous seed)."""
        ctx = self.gen.ctx
        tm = timer or (lambda name: _NullCtx())
        if seed is not None:
            check(ctx.lib.pods_df_set_seed(ctx.h, int(seed) & 0xffffffff), "pods_df_set_seed")
        bank = self.k % 2 if self.pipelined else 0
        check(ctx.lib.pods_select_snapshots(ctx.h, bank), "pods_select_snapshots")
        if prefetch_next and os.environ.get("PODS_JUMP_EARLY", "1") != "0":
            self.gen.prefetch_jump_early(timer)   # the next step's jump beside this generation
        with tm("generate"):
            snap = self.gen.generate()
        if prefetch_next:
            self.gen.prefetch_jump(timer)
        C, mean = pod_head(snap, self.world, timer, partial=self.collectives)
        # without a collective nothing else orders rank 0's solve stream behind this correlation
        c_done = None
        if not self.collectives:
            c_done = torch.cuda.Event()
            c_done.record()
        if self.pending is not None:
            self._tail(timer)
        check(ctx.lib.pods_select_snapshots(ctx.h, bank), "pods_select_snapshots")
        finish = None
        if self.collectives:
            if self.world > 1:
                ctx.detect_sharing(self.dist)
            # the packed partial C goes out now; with the pipeline the main stream does not wait for
            # it (the next step's generation runs beside the all-reduce) -- its tail unpacks it
            pack, unpack = device_triangle_ops(ctx)
            with tm("allreduce"):
                packed = pack(C)
                work = self.dist.all_reduce(packed, async_op=True)

            def finish(packed=packed, work=work, unpack=unpack, C=C):
                # on whatever stream is current (rank 0's tail: its solve stream)
                work.wait()
                packed.record_stream(torch.cuda.current_stream(ctx.device))
                unpack(packed, C)
        self.pending = [bank, snap, C, mean, finish, c_done]
        self.k += 1
        if not self.pipelined:
            self._tail(timer)

    def _tail(self, timer):
        bank, snap, C, mean, finish, c_done = self.pending
        self.pending = None
        ctx = self.gen.ctx
        solve = self._solve_stream() if self.rank == 0 else None
        ready = None
        if solve is not None:
            # rank 0: the leading-pair solve of step k-1 depends on step k-1's all-reduce only, so
            # the finisher (RCCL: the solve stream waits for the collective) and the unpack go to
            # the solve stream, which then runs beside step k's generation and correlation on the
            # main stream (an event recorded on the main stream here used to order the
            # solve behind step k's correlation).  Before it: the spectrum units this rank enqueued
            # on the main stream in earlier tails (persistent k_trd grids: nothing may take their
            # CUs while they run).  The solve's own kernels (subspace iteration) are not persistent:
            # beside the generator and the paced SYRK they only share the CUs.
            if self._spec_done is not None:
                solve.wait_event(self._spec_done)
            if c_done is not None:   # no collective: the correlation itself, on the main stream
                solve.wait_event(c_done)
            with ctx.on_stream(solve):
                if finish is not None:
                    finish()
                C.record_stream(solve)
                ready = torch.cuda.Event()
                ready.record(solve)
            # the main stream reads C later (this rank's spectrum units, after the solve)
            torch.cuda.current_stream(ctx.device).wait_event(ready)
        elif finish is not None:
            finish()   # the main stream waits for this step's all-reduce, then unpacks C
        s = self.setup
        self.gen.join_ahead()   # the persistent spectrum kernels must not find generator workgroups
        check(ctx.lib.pods_select_snapshots(ctx.h, bank), "pods_select_snapshots")
        fo = []

        def start_fourier(T, nmt, t_ready):
            fo.append(launch_fourier(ctx, T, nmt, s.ns, s.dt_eff, s.et, timer=timer, side=True, ready=t_ready))
        if self.backlog is not None:
            self.backlog.finish_pending()
        pod = pod_tail(ctx, snap, C, mean, s.nm, 1.0e-15, self.dist, timer=timer, on_temporal=start_fourier,
                       spectrum=self.spectrum, solve_stream=solve, c_ready=ready)
        # everything pod_tail put on the main stream (this rank's spectrum units among it): the next
        # tail's solve starts behind it
        self._spec_done = torch.cuda.Event()
        self._spec_done.record()
        self.results.append(pod)
        if self.backlog is not None:
            self.backlog.pending.append(fo[-1] if fo else None)

    def flush(self, timer=None):
        if self.pending is not None:
            self._tail(timer)
        if self.backlog is not None:
            self.backlog.finish_pending()


def wall():
    return time.perf_counter()
