"""Host-side problem setup of the digital-filter path (small, O(P) work, numpy).

These are the reference's per-run host computations, kept on the host because they
are tiny and must be bit-identical to the reference:
  calccoeff            digitalfilters.py:73-89
  build_profile        digitalfilters.py:1038-1062
  adapt1d factor       digitalfilters.py:151-172  (per k, evaluated once per run)
  adapt2prf factor     digitalfilters.py:187-222  (per point, evaluated once per run)
  prof_rotation_matrix digitalfilters.py:1064-1116
  main() option logic  digitalfilters.py:1244-1322 (nf, dt / anisotropic lnx, clamps)
The per-step work (filters, Lund application, rotation) runs on the GPU.
"""
import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

SQRT3 = np.sqrt(3.0)


def calccoeff(n, ln):
    a = np.zeros(n * 2 + 1)
    norm = 0.0
    for i in range(n * 2 + 1):
        k = float(i - n)
        a[i] = np.exp(-np.pi * k * k / (2.0 * ln * ln))
        norm = norm + a[i] ** 2
    return a / np.sqrt(norm)


def build_profile(mean_profile, turb_profile, bulk_velocity, turbulence_intensity, kma):
    if mean_profile in ("hyperbolic-tangent", "double-hyperbolic-tangent",
                        "circular-hyperbolic-tangent", "ring-hyperbolic-tangent"):
        y = np.linspace(-0.5, 0.5, kma)
        U = bulk_velocity / 2 * (1. + np.tanh(10. * (-np.abs(y) + 0.5)))
    else:
        raise Exception("Invalid mean_profile chosen, type 'python digitalfilters.py -h' for help.")
    if turb_profile == "top-hat":
        uu = (turbulence_intensity * U) ** 2
        vv = (turbulence_intensity * U) ** 2
        ww = (turbulence_intensity * U) ** 2
        uw = 0.0 * U
    elif turb_profile == "none":
        uu = vv = ww = uw = 0.0
    else:
        raise Exception("Invalid turb_profile chosen, type 'python digitalfilters.py -h' for help.")
    return U, uu, vv, ww, uw


def lund1d_factor(uu, vv, ww, uw):
    """adapt1d's lower-triangular factor per k (R10 = R21 = 0, +1e-20 guards)."""
    uu, vv, ww, uw = (np.asarray(v, dtype=np.float64) for v in (uu, vv, ww, uw))
    zero = np.zeros_like(uu)
    with np.errstate(invalid="ignore"):
        a00 = np.sqrt(uu)
        a10 = zero / (a00 + 1e-20)
        a11 = np.sqrt(vv - a10 * a10)
        a20 = uw / (a00 + 1e-20)
        a21 = (zero - a10 * a20) / (a11 + 1e-20)
        a22 = np.sqrt(ww - a20 * a20 - a21 * a21)
    return a00, a10, a11, a20, a21, a22


def lundprf_factor(uu, vv, ww, uv, uw, vw):
    """adapt2prf's guarded factor per point."""
    uu, vv, ww, uv, uw, vw = (np.asarray(v, dtype=np.float64) for v in (uu, vv, ww, uv, uw, vw))
    with np.errstate(invalid="ignore", divide="ignore"):
        a00 = np.sqrt(uu)
        a10 = np.where(a00 > 0., uv / (a00 + 1e-20), 0.0)
        neg = a10 ** 2 > vv
        a11 = np.where(neg, 0.0, np.sqrt(np.where(neg, 0.0, vv - a10 * a10)))
        a20 = np.where(a00 > 0.0, uw / (a00 + 1e-20), 0.0)
        a21 = np.where(a11 > 0.0, (vw - a10 * a20) / (a11 + 1e-20), 0.0)
        neg = ww < a20 * a20 + a21 * a21
        a22 = np.where(neg, 0.0, np.sqrt(np.where(neg, 0.0, ww - a20 * a20 - a21 * a21)))
    return a00, a10, a11, a20, a21, a22


PROFILES_2D = ("double-hyperbolic-tangent", "circular-hyperbolic-tangent", "ring-hyperbolic-tangent")


def _adapt2d_lund(R00, R11, R22, R20):
    """adapt2d's clamped factor (digitalfilters.py:278-299, same at :365-385 and :457-477).
    R10 = R21 = 0 (never assigned; R starts zero); A00 = sqrt(R00) is NOT clamped (the
    clamped temp1 above it is unused), so a negative R00 gives NaN exactly like the reference."""
    zero = np.zeros_like(R00)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        a00 = np.sqrt(R00)
        a10 = zero / (a00 + 1e-20)
        t = R11 - a10 * a10
        a11 = np.sqrt(np.where(t < 0, 0.0, t))
        a20 = R20 / (a00 + 1e-20)
        a21 = (zero - a10 * a20) / (a11 + 1e-20)
        t = R22 - a20 * a20 - a21 * a21
        a22 = np.sqrt(np.where(t < 0, 0.0, t))
    return a00, a10, a11, a20, a21, a22


def prof_rotation_matrix(nx, ny, nz):
    n = np.sqrt(nx ** 2 + ny ** 2 + nz ** 2)
    n_proj = np.sqrt(nx ** 2 + ny ** 2)
    if ny > 0:
        azimuth = np.arccos(nx / n_proj)
    elif ny < 0:
        azimuth = -np.arccos(nx / n_proj)
    elif ny == 0 and nx >= 0:
        azimuth = 0.
    else:
        azimuth = np.pi
    c, s = np.cos(azimuth), np.sin(azimuth)
    Ra = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    if nz > 0:
        polar = np.arccos(n_proj / n)
    elif nz < 0:
        polar = -np.arccos(n_proj / n)
    else:
        polar = 0.
    c, s = np.cos(polar), np.sin(polar)
    Rp = np.array([[c, 0, -s], [0, 1, 0], [s, 0, c]])
    return Ra.dot(Rp)


@dataclass
class DFSetup:
    """Everything main() derives from its options before the step loop."""
    jma: int
    kma: int
    ns: int
    seed: int = 12345
    lengthscale: float = 3.0
    fwidth: float = 2.0
    dt: float = 0.0
    res: float = 0.1
    bulk_velocity: float = 1.0
    u_dash: float = 0.02
    nm: int = 20
    et: float = 0.9
    normal: tuple = (1.0, 0.0, 0.0)
    mean_profile: str = "hyperbolic-tangent"
    turb_profile: str = "top-hat"
    inner_d: float = 0.5                # --ring (:1275): inner radius of the ring profile
    ln_prf: Optional[float] = None      # lnx = lny = lnz returned by read_prf (:1301-1305)
    prf: Optional[dict] = None         # (jma,kma) arrays U,V,W,uu,vv,ww,uv,uw,vw -> adapt2prf
    profile1d: Optional[dict] = None    # (kma,) arrays U,uu,vv,ww,uw from read_profile -> adapt1d
    nfx: int = field(default=0, init=False)
    nfy: int = field(default=0, init=False)
    nfz: int = field(default=0, init=False)
    lnx: float = field(default=0.0, init=False)
    lny: float = field(default=0.0, init=False)
    lnz: float = field(default=0.0, init=False)
    dt_eff: float = field(default=0.0, init=False)
    n_unit: tuple = field(default=(), init=False)
    profile: dict = field(default_factory=dict, init=False)

    def __post_init__(self):
        self.lnx = self.lny = self.lnz = float(self.lengthscale)
        nf = int(math.ceil(self.fwidth * self.lengthscale))  # :1282, from the CLI length scale
        self.nfx = self.nfy = self.nfz = nf
        if self.ln_prf is not None:  # a .prf file replaces the taps' length scale, not nf
            self.lnx = self.lny = self.lnz = float(self.ln_prf)
        n1 = np.asarray(self.normal, dtype=np.float64)
        nrm = np.sqrt(n1[0] ** 2 + n1[1] ** 2 + n1[2] ** 2)
        self.n_unit = (n1[0] / nrm, n1[1] / nrm, n1[2] / nrm)
        V = W = 0
        if self.prf is None and self.profile1d is not None:
            self.profile = {k: np.array(self.profile1d[k], dtype=np.float64) for k in ("U", "uu", "vv", "ww", "uw")}
            U = self.profile["U"]
        elif self.prf is None:
            U, uu, vv, ww, uw = build_profile(self.mean_profile, self.turb_profile,
                                              self.bulk_velocity, self.u_dash, self.kma)
            self.profile = dict(U=np.asarray(U, dtype=np.float64), uu=uu, vv=vv, ww=ww, uw=uw)
        else:
            self.profile = {k: np.asarray(v, dtype=np.float64) for k, v in self.prf.items()}
            U, V, W = self.profile["U"], self.profile["V"], self.profile["W"]
        flag = np.where(U ** 2 + V ** 2 + W ** 2 != 0)
        if self.dt == 0.:
            self.dt_eff = self.res / np.mean(U[flag])
        else:
            dt1 = self.res / np.mean(U[flag])
            factor = dt1 / self.dt
            self.lnx = factor * self.lnx
            self.nfx = int(math.ceil(float(self.fwidth) * self.lnx))
            self.dt_eff = self.dt
        if self.prf is None:
            for key in ("uu", "vv", "ww"):
                arr = self.profile[key]
                if np.ndim(arr):
                    arr[arr < 0.0] = 0.0

    @property
    def P(self):
        return self.jma * self.kma

    @property
    def rotated(self):
        """main() rotates only when the profile was built, not read (:1476)."""
        return self.prf is None and self.profile1d is None

    def taps(self):
        return (calccoeff(self.nfx, self.lnx), calccoeff(self.nfy, self.lny),
                calccoeff(self.nfz, self.lnz))

    def rotation(self):
        return prof_rotation_matrix(*self.n_unit)

    def lund_mode(self):
        return 0 if self.prf is None else 1

    def lund_rows(self, j0=0, j1=None):
        """(9, P_slab) SoA: a00,a10,a11,a20,a21,a22,U,V,W for rows [j0, j1)."""
        j1 = self.jma if j1 is None else j1
        J, K = self.jma, self.kma
        pr = self.profile
        out = np.zeros((9, J, K))
        if self.prf is None and self.mean_profile in PROFILES_2D:
            # main() :1447-1449: adapt2d for the 2-D built (or 1-D file) profiles
            from .profiles2d import adapt2d_factor
            fac = adapt2d_factor(self.mean_profile, self.inner_d, pr["U"], pr["uu"], pr["vv"], pr["ww"],
                                 pr["uw"], J, K)
            for r in range(7):
                out[r] = fac[r]
        elif self.prf is None:
            fac = lund1d_factor(*(np.broadcast_to(np.asarray(pr[k], dtype=np.float64), (K,))
                                  for k in ("uu", "vv", "ww", "uw")))
            for r, v in enumerate(fac):
                out[r] = np.broadcast_to(np.asarray(v, dtype=np.float64), (K,))[None, :]
            out[6] = pr["U"][None, :]
        else:
            fac = lundprf_factor(pr["uu"], pr["vv"], pr["ww"], pr["uv"], pr["uw"], pr["vw"])
            for r, v in enumerate(fac):
                out[r] = v
            out[6], out[7], out[8] = pr["U"], pr["V"], pr["W"]
        return np.ascontiguousarray(out[:, j0:j1, :].reshape(9, (j1 - j0) * K))


def row_slab(jma, rank, world):
    """Contiguous row slab [j0, j1) of rank `rank` among `world`."""
    base, extra = divmod(jma, world)
    j0 = rank * base + min(rank, extra)
    return j0, j0 + base + (1 if rank < extra else 0)


def time_axis(ns, dt):
    """PODFS.py:1540-1542."""
    time = np.linspace(0, (ns - 1) * dt * 1, ns)
    period = time[-1] + (time[1] - time[0]) if ns > 1 else dt
    return time, period


def dft_rows(ns):
    """The k of each twiddle-table row (pods_fourier_twiddles): k = 0..nk-1 and, for even ns,
    k = -ns/2 (the n = 0 coefficient); the negative k of the other n are exact conjugates."""
    h = ns // 2
    nk = h if ns % 2 == 0 else h + 1
    return list(range(nk)) + ([-h] if ns % 2 == 0 else [])


def dft_twiddles(ns, time, period, chunk=128):
    """np.exp(-1j*2*k*np.pi*time/period) for every table row k -- the reference's own
    expression (PODFS.py:1566, with k = n - num_fcs/2), evaluated by numpy on the host so the
    GPU DFT multiplies by exactly the numbers the reference does.  Rows are evaluated in
    chunks as (coef[:, None] * time) / period: the same complex128 ufunc loops, element for
    element, as the per-k expression (tests/test_host_cpu.py pins the bits).
    Returns an (R, ns, 2) float64 array of (cos, sin)."""
    ks = dft_rows(ns)
    time = np.asarray(time, dtype=np.float64)
    W = np.empty((len(ks), ns, 2), dtype=np.float64)

    def rows(r0):
        coef = np.array([-1j * 2 * k * np.pi for k in ks[r0:r0 + chunk]], dtype=np.complex128)
        E = np.exp(coef[:, None] * time[None, :] / period)
        W[r0:r0 + len(coef), :, 0] = E.real
        W[r0:r0 + len(coef), :, 1] = E.imag
    starts = list(range(0, len(ks), chunk))
    if len(starts) > 1:  # numpy releases the GIL inside the ufunc loops
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(8, len(starts))) as ex:
            list(ex.map(rows, starts))
    else:
        rows(0)
    return W


def num_valid_modes_loop(energy, ns, tol_CN=1.0e-15):
    """PODFS.py:1312-1317, literally (a Python loop over up to ns - 2 numpy scalars)."""
    n = 0
    while ((energy[n] / energy[0] > pow(tol_CN, 2.0)) and (n < ns - 2) and (energy[n] > 0.0)):
        n += 1
        if (energy[n] / energy[0] > pow(tol_CN, 2.0)) and (energy[n] > 0.0):
            n += 1
    return n


def num_valid_modes(energy, ns, tol_CN=1.0e-15):
    """PODFS.py:1312-1317 without the Python loop (0.9 ms at ns = 4096): the loop tests
    cond(i) = energy[i]/energy[0] > tol^2 and energy[i] > 0 at even positions and steps by
    two while cond holds at both, so it stops at the first index f where cond fails, or at
    the first even position E >= ns - 2 where the bound stops it: the result is min(f, E).
    The same per-element arithmetic as the loop; pinned against num_valid_modes_loop."""
    e = np.asarray(energy)
    if ns < 1 or e.shape[0] < 1:
        return 0
    bound = ns - 2
    E = max(bound + (bound & 1), 0)
    m = min(E + 1, e.shape[0])
    head = e[:m]
    with np.errstate(divide="ignore", invalid="ignore"):
        cond = (head / head[0] > pow(tol_CN, 2.0)) & (head > 0.0)
    bad = np.flatnonzero(~cond)
    f = int(bad[0]) if bad.size else m
    return min(f, E)


def rank_and_count(c, et):
    """PODFS.py:1575-1593 on one complex64 column: order by (|c| f32, n) descending
    (sorted(zip(cmod, idx), reverse=True)); count coefficients until the float64 running
    sum of |c| reaches float64(sum_f32 |c|) * et (Python 2 / numpy-1.x promotion)."""
    ns = len(c)
    cmod = np.abs(c)
    order = np.lexsort((np.arange(ns), cmod))[::-1].astype(np.int32)
    target = np.float64(np.sum(np.abs(c))) * et
    if not target > 0.0:
        return order, 0
    # np.cumsum in float64 is the same left-to-right accumulation as the reference's
    # `energy += ...` loop, so csum[i] is bit-identical to `energy` after i+1 additions.
    csum = np.cumsum(cmod[order].astype(np.float64))
    hit = int(np.searchsorted(csum, target, side="left"))
    if hit >= ns:
        raise IndexError("energy target %r not reachable (et > 1?)" % et)
    return order, hit + 1
