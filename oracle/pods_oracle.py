"""CPU oracle: a numpy/scipy restatement of the reference's digital-filter + PODFS path.

TEST INFRASTRUCTURE.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker or as the timed CPU
baseline.  The product (pods-digital-filter_amd/) never imports it.

Pinning: every function below is checked bit-for-bit against fixtures produced by
running the reference's own functions (tests/golden/make_golden.py, which executes
digitalfilters.py / PODFS.py code translated in memory).  See tests/test_oracle_golden.py.

Each function cites the reference file:line it restates.  Two kinds of function live here:

* reference-call restatements (generate, pod, fourier ...) that make the same numpy /
  scipy calls as the reference, in the same order -> bit-identical by construction;
* explicit restatements of numpy/scipy *internals* that the GPU kernels replicate
  (filter_block's summation order == scipy _correlateND direct path; pairwise_sum /
  cpairwise_sum == numpy's pairwise summation; dft_explicit == numpy's complex
  expression at PODFS.py:1566).  These are pinned against the library calls.

`loops=True` variants reproduce the reference's per-point Python loops (adapt1d,
rotate_velocity, the y2 reconstruction loop) so the CPU baseline is timed on the same
work the reference does.
"""
import math
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

try:  # scipy is the reference's own dependency (digitalfilters.py:23)
    import scipy.signal as _scsig
except Exception:  # pragma: no cover
    _scsig = None

SQRT3 = np.sqrt(3.0)


# ----------------------------------------------------------------------------------------
# filter taps, profiles, Lund transform, rotation
# ----------------------------------------------------------------------------------------
def calccoeff(n, ln):
    """digitalfilters.py:73-89 -- b_i = exp(-pi k^2 / (2 ln^2)) / sqrt(sum b^2), sequential norm."""
    a = np.zeros(2 * n + 1)
    norm = 0.0
    for i in range(n * 2 + 1):
        k = float(i - n)
        a[i] = np.exp(-np.pi * k * k / (2.0 * ln * ln))
        norm = norm + a[i] ** 2
    return a / np.sqrt(norm)


def build_profile(mean_profile, turb_profile, bulk_velocity, turbulence_intensity, kma):
    """digitalfilters.py:1038-1062."""
    if mean_profile not in ("hyperbolic-tangent", "double-hyperbolic-tangent",
                            "circular-hyperbolic-tangent", "ring-hyperbolic-tangent"):
        raise ValueError("Invalid mean_profile chosen")
    y = np.linspace(-0.5, 0.5, kma)
    U = bulk_velocity / 2 * (1. + np.tanh(10. * (-np.abs(y) + 0.5)))
    if turb_profile == "top-hat":
        uu = (turbulence_intensity * U) ** 2
        vv = (turbulence_intensity * U) ** 2
        ww = (turbulence_intensity * U) ** 2
        uw = 0.0 * U
    elif turb_profile == "none":
        uu = vv = ww = uw = 0.0
    else:
        raise ValueError("Invalid turb_profile chosen")
    return U, uu, vv, ww, uw


def lund1d_coeffs(uu, vv, ww, uw):
    """adapt1d's per-k Cholesky factor, digitalfilters.py:151-172.  Arrays over k.
    R10 = R21 = 0 (never assigned; R starts zero).  Returns a00,a10,a11,a20,a21,a22."""
    uu, vv, ww, uw = (np.asarray(v, dtype=np.float64) for v in (uu, vv, ww, uw))
    R10 = np.zeros_like(uu)
    R21 = np.zeros_like(uu)
    with np.errstate(invalid="ignore"):
        a00 = np.sqrt(uu)
        a10 = R10 / (a00 + 1e-20)
        a11 = np.sqrt(vv - a10 * a10)
        a20 = uw / (a00 + 1e-20)
        a21 = (R21 - a10 * a20) / (a11 + 1e-20)
        a22 = np.sqrt(ww - a20 * a20 - a21 * a21)
    return a00, a10, a11, a20, a21, a22


def lundprf_coeffs(uu, vv, ww, uv, uw, vw):
    """adapt2prf's guarded per-point Cholesky factor, digitalfilters.py:187-222."""
    uu, vv, ww, uv, uw, vw = (np.asarray(v, dtype=np.float64) for v in (uu, vv, ww, uv, uw, vw))
    with np.errstate(invalid="ignore", divide="ignore"):
        a00 = np.sqrt(uu)
        a10 = np.where(a00 > 0., uv / (a00 + 1e-20), 0.0)
        a11 = np.where(a10 ** 2 > vv, 0.0, np.sqrt(np.where(a10 ** 2 > vv, 0.0, vv - a10 * a10)))
        a20 = np.where(a00 > 0.0, uw / (a00 + 1e-20), 0.0)
        a21 = np.where(a11 > 0.0, (vw - a10 * a20) / (a11 + 1e-20), 0.0)
        cond = ww < a20 * a20 + a21 * a21
        a22 = np.where(cond, 0.0, np.sqrt(np.where(cond, 0.0, ww - a20 * a20 - a21 * a21)))
    return a00, a10, a11, a20, a21, a22


def apply_lund(yu, yv, yw, coeffs, U, V=None, W=None):
    """u = a00 xu + 0 xv + 0 xw + U ; v = a10 xu + a11 xv + 0 xw (+V) ; w = a20 xu + a21 xv + a22 xw (+W)
    evaluated left to right with the zero terms included (digitalfilters.py:174-178, :227-231).
    V/W None -> adapt1d form (no mean added to v, w)."""
    a00, a10, a11, a20, a21, a22 = coeffs
    xu, xv, xw = yu.copy(), yv.copy(), yw.copy()
    u = a00 * xu + 0.0 * xv + 0.0 * xw + U
    v = a10 * xu + a11 * xv + 0.0 * xw
    w = a20 * xu + a21 * xv + a22 * xw
    if V is not None:
        v = v + V
        w = w + W
    return u, v, w


def adapt1d_loops(yu, yv, yw, uin, uuin, vvin, wwin, uwin, jma, kma):
    """Reference-faithful Python loop form of adapt1d (digitalfilters.py:143-178), CPU baseline only."""
    R = np.zeros((3, 3))
    A = np.zeros((3, 3))
    for k in range(kma):
        R[0, 0] = uuin[k]; R[1, 1] = vvin[k]; R[2, 2] = wwin[k]; R[2, 0] = uwin[k]
        A[:, :] = 1.0
        A[0, 0] = np.sqrt(R[0, 0]); A[0, 1] = 0.0; A[0, 2] = 0.0
        A[1, 0] = R[1, 0] / (A[0, 0] + 1e-20)
        A[1, 1] = np.sqrt(R[1, 1] - A[1, 0] * A[1, 0]); A[1, 2] = 0.0
        A[2, 0] = R[2, 0] / (A[0, 0] + 1e-20)
        A[2, 1] = (R[2, 1] - A[1, 0] * A[2, 0]) / (A[1, 1] + 1e-20)
        A[2, 2] = np.sqrt(R[2, 2] - A[2, 0] * A[2, 0] - A[2, 1] * A[2, 1])
        for j in range(jma):
            xu = yu[j, k]; xv = yv[j, k]; xw = yw[j, k]
            yu[j, k] = A[0, 0] * xu + A[0, 1] * xv + A[0, 2] * xw + uin[k]
            yv[j, k] = A[1, 0] * xu + A[1, 1] * xv + A[1, 2] * xw
            yw[j, k] = A[2, 0] * xu + A[2, 1] * xv + A[2, 2] * xw


PROFILES_2D = ("double-hyperbolic-tangent", "circular-hyperbolic-tangent", "ring-hyperbolic-tangent")


def _clamped_factor(R00, R11, R22, R20):
    """adapt2d's factor for one point (digitalfilters.py:278-299 / :365-385 / :457-477):
    R10 = R21 = 0; A00 = sqrt(R00) unclamped (the clamped temp1 before it is never used)."""
    A = np.ones((3, 3))
    A[0, 0] = np.sqrt(R00)
    A[0, 1] = 0.0
    A[0, 2] = 0.0
    A[1, 0] = 0.0 / (A[0, 0] + 1e-20)
    t = R11 - A[1, 0] * A[1, 0]
    if t < 0:
        t = 0.0
    A[1, 1] = np.sqrt(t)
    A[1, 2] = 0.0
    A[2, 0] = R20 / (A[0, 0] + 1e-20)
    A[2, 1] = (0.0 - A[1, 0] * A[2, 0]) / (A[1, 1] + 1e-20)
    t = R22 - A[2, 0] * A[2, 0] - A[2, 1] * A[2, 1]
    if t < 0:
        t = 0.0
    A[2, 2] = np.sqrt(t)
    return A


def adapt2d_point_coeffs(mean_profile, inner_d, uin, uuin, vvin, wwin, uwin, jma, kma):
    """adapt2d (digitalfilters.py:233-485) evaluated point by point with scalar splev, as the
    reference does inside its step loop.  Returns ((a00,a10,a11,a20,a21,a22), Umean), (J, K)
    arrays; the transform itself is apply_lund with these per-point factors (V/W None)."""
    from scipy import interpolate
    J, K = jma, kma
    prof = [np.array(np.broadcast_to(np.asarray(v, dtype=np.float64), (K,))) for v in (uin, uuin, vvin, wwin, uwin)]
    co = np.zeros((6, J, K))
    um = np.zeros((J, K))
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if mean_profile == "double-hyperbolic-tangent":                  # :238-307
            zA = np.linspace(-1., 1, K)
            zi = np.linspace(-1., 1, J)
            inj = [interpolate.splev(zi, interpolate.splrep(zA, v, s=0), der=0) for v in prof]
            for v, src in zip(inj, prof):
                v[0], v[-1] = src[0], src[-1]
            for j in range(J):
                for v in inj[1:4]:
                    if v[j] < 0.:
                        v[j] = 0.0
                for k in range(K):
                    R00 = np.sqrt(prof[1][k] * inj[1][j])
                    R11 = np.sqrt(prof[2][k] * inj[2][j])
                    R22 = np.sqrt(prof[3][k] * inj[3][j])
                    R20 = np.sign(prof[4][k] + inj[4][j]) * np.sqrt(abs(prof[4][k] * inj[4][j]))
                    A = _clamped_factor(R00, R11, R22, R20)
                    co[:, j, k] = (A[0, 0], A[1, 0], A[1, 1], A[2, 0], A[2, 1], A[2, 2])
                    um[j, k] = np.sqrt(prof[0][k] * inj[0][j])
        elif mean_profile in ("circular-hyperbolic-tangent", "ring-hyperbolic-tangent"):
            x = np.linspace(-1., 1., J)
            y = np.linspace(-1., 1., K)
            ring = mean_profile == "ring-hyperbolic-tangent"
            if ring:                                                     # :395-485
                zA = np.linspace(inner_d, 1., K)
                tck = [interpolate.splrep(zA, v, s=0) for v in prof]
                r_lo, lo = inner_d, [v[0] for v in prof]
            else:                                                        # :309-393
                ci = np.argmax(prof[0])
                zA = np.linspace(0, 1, len(prof[0]) - ci)
                tck = [interpolate.splrep(zA, v[ci:], s=0) for v in prof]
                r_lo, lo = 0.0, [v[ci] for v in prof]
            for j in range(J):
                for k in range(K):
                    r = np.sqrt(x[j] ** 2 + y[k] ** 2)
                    val = [interpolate.splev(r, t, der=0) for t in tck]
                    if r == r_lo:
                        val = list(lo)
                    if r == 1.0:
                        val = [v[-1] for v in prof]
                    if r > 1.0:
                        val = [0.0] * 5
                    if ring and r < inner_d:
                        val = [0.0] * 5
                    A = _clamped_factor(val[1], val[2], val[3], val[4])
                    co[:, j, k] = (A[0, 0], A[1, 0], A[1, 1], A[2, 0], A[2, 1], A[2, 2])
                    um[j, k] = val[0]
        else:
            raise ValueError("adapt2d: unknown mean_profile %r" % (mean_profile,))
    return tuple(co), um


def read_profile(path, kma):
    """read_profile (digitalfilters.py:487-522): columns y, U, uu, vv, ww, uv; the half-channel
    rows are mirrored about y = 1 (uv changes sign), y normalised to [0, 1], each column
    interpolated to kma points with an interpolating cubic spline, both walls set to zero."""
    from scipy import interpolate
    d = np.genfromtxt(path, names=True, autostrip=True, comments="#")
    n = d.shape[0]
    mirrored = d[0:n - 2][::-1]
    d = np.concatenate([d, mirrored])
    d["y"][n:] = (-(d["y"][n:] - 1.0) + 1)
    d["uv"][n:] = -d["uv"][n:]
    z = d["y"]
    z = (z - np.min(z)) / (np.max(z) - np.min(z))
    zi = np.linspace(np.min(z), np.max(z), kma)
    out = []
    for name in ("U", "uu", "vv", "ww", "uv"):
        v = interpolate.splev(zi, interpolate.splrep(z, d[name], s=0), der=0)
        v[0] = v[-1] = 0.
        out.append(v)
    return tuple(out)


def rotation_matrix(nx, ny, nz):
    """prof_rotation_matrix, digitalfilters.py:1064-1116 (R = Ra(azimuth) . Rp(polar))."""
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


def rotate_velocity(Acol, R):
    """rotate_velocity, digitalfilters.py:1119-1131 -- per point R.dot(V) (numpy dot)."""
    pts = len(Acol) // 3
    out = np.zeros(len(Acol))
    for i in range(pts):
        V = np.array([Acol[i], Acol[i + pts], Acol[i + 2 * pts]])
        Vr = R.dot(V)
        out[i], out[i + pts], out[i + 2 * pts] = Vr[0], Vr[1], Vr[2]
    return out


# ----------------------------------------------------------------------------------------
# the separable filter: scipy direct-path summation order, restated
# ----------------------------------------------------------------------------------------
def filter_block(x, bx, by, bz):
    """filter3DSciPy1D (digitalfilters.py:100-140) restated with scipy's direct-path order:
    three 'valid' passes x -> y -> z, each acc = 0.0; acc += in[i+a]*b[2n-a], a ascending
    (scipy _correlateND with the reversed, symmetric kernel).  Bit-identical to scipy."""
    nxa, nya, nza = len(bx), len(by), len(bz)
    J = x.shape[1] - nya + 1
    K = x.shape[2] - nza + 1
    acc = np.zeros(x.shape[1:])
    for a in range(nxa):
        acc = acc + x[a] * bx[nxa - 1 - a]
    t1 = acc
    acc = np.zeros((J, x.shape[2]))
    for b in range(nya):
        acc = acc + t1[b:b + J] * by[nya - 1 - b]
    t2 = acc
    acc = np.zeros((J, K))
    for c in range(nza):
        acc = acc + t2[:, c:c + K] * bz[nza - 1 - c]
    return acc


def filter_block_scipy(x, bx, by, bz):
    """The reference's literal call sequence (digitalfilters.py:124-140)."""
    t1 = _scsig.convolve(x, bx[:, None, None], mode="valid", method="direct")
    t2 = _scsig.convolve(t1, by[None, :, None], mode="valid", method="direct")
    t3 = _scsig.convolve(t2, bz[None, None, :], mode="valid", method="direct")
    return t3[0]


# ----------------------------------------------------------------------------------------
# numpy pairwise summation (the order np.mean / ndarray.sum use), restated
# ----------------------------------------------------------------------------------------
PW_BLOCKSIZE = 128
NPY_BUFSIZE = 8192


def pairwise_program(n):
    """Post-order program for numpy's real pairwise sum of n items (numpy loops_utils
    pairwise_sum): list of ('leaf', start, length) and ('add',) ops.  The GPU mean
    kernel interprets exactly this program."""
    prog = []

    def rec(start, m):
        if m <= PW_BLOCKSIZE:
            prog.append(("leaf", start, m))
            return
        m2 = m // 2
        m2 -= m2 % 8
        rec(start, m2)
        rec(start + m2, m - m2)
        prog.append(("add",))

    # numpy's reduction iterator hands the inner loop at most NPY_BUFSIZE (8192) items at
    # a time and accumulates the chunk sums left to right.
    for s in range(0, n, NPY_BUFSIZE):
        rec(s, min(NPY_BUFSIZE, n - s))
        if s:
            prog.append(("add",))
    return prog


def pairwise_leaf(a):
    n = len(a)
    if n < 8:
        res = 0.0
        for v in a:
            res += v
        return res
    r = [a[j] for j in range(8)]
    i = 8
    while i < n - (n % 8):
        for j in range(8):
            r[j] += a[i + j]
        i += 8
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    while i < n:
        res += a[i]
        i += 1
    return res


def pairwise_sum(a):
    """Explicit numpy pairwise sum of a 1-D float64 sequence (== np.add.reduce)."""
    a = np.asarray(a, dtype=np.float64)
    stack = []
    for op in pairwise_program(len(a)):
        if op[0] == "leaf":
            stack.append(pairwise_leaf(a[op[1]:op[1] + op[2]]))
        else:
            b = stack.pop()
            stack.append(stack.pop() + b)
    return 0.0 + stack[0] if stack else 0.0


def cpairwise_program(n):
    """Post-order program for numpy's complex pairwise sum over n complex items
    (CDOUBLE_pairwise_sum works in half-units: leaf when 2n <= 128, split at
    (2n/2 - (2n/2)%8) half-units)."""
    prog = []

    def rec(start, m):
        if 2 * m <= PW_BLOCKSIZE:
            prog.append(("leaf", start, m))
            return
        h = m  # (2m)/2 half units
        h -= h % 8
        m2 = h // 2
        rec(start, m2)
        rec(start + m2, m - m2)
        prog.append(("add",))

    for s in range(0, n, NPY_BUFSIZE):
        rec(s, min(NPY_BUFSIZE, n - s))
        if s:
            prog.append(("add",))
    return prog


def cpairwise_leaf(re, im):
    n = len(re)
    if n < 4:
        rr, ri = -0.0, -0.0
        for i in range(n):
            rr += re[i]
            ri += im[i]
        return rr, ri
    r = [re[0], im[0], re[1], im[1], re[2], im[2], re[3], im[3]]
    i = 4
    while i < n - (n % 4):
        r[0] += re[i]; r[1] += im[i]; r[2] += re[i + 1]; r[3] += im[i + 1]
        r[4] += re[i + 2]; r[5] += im[i + 2]; r[6] += re[i + 3]; r[7] += im[i + 3]
        i += 4
    rr = (r[0] + r[2]) + (r[4] + r[6])
    ri = (r[1] + r[3]) + (r[5] + r[7])
    while i < n:
        rr += re[i]
        ri += im[i]
        i += 1
    return rr, ri


def cpairwise_sum(re, im):
    stack = []
    for op in cpairwise_program(len(re)):
        if op[0] == "leaf":
            s, m = op[1], op[2]
            stack.append(cpairwise_leaf(re[s:s + m], im[s:s + m]))
        else:
            b = stack.pop()
            a = stack.pop()
            stack.append((a[0] + b[0], a[1] + b[1]))
    return stack[0]


# ----------------------------------------------------------------------------------------
# configuration (mirrors main()'s option handling, digitalfilters.py:1244-1322)
# ----------------------------------------------------------------------------------------
@dataclass
class DFConfig:
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
    prf: Optional[dict] = None
    mean_profile: str = "hyperbolic-tangent"   # -p (:1146); the 2-D ones go through adapt2d
    inner_d: float = 0.5                       # --ring (:1275)
    ln_prf: Optional[float] = None             # lnx from read_prf (:1301-1305)
    profile1d: Optional[dict] = None           # U,uu,vv,ww,uw from read_profile (:1306-1307)
    # derived
    nfx: int = 0
    nfy: int = 0
    nfz: int = 0
    lnx: float = 0.0
    lny: float = 0.0
    lnz: float = 0.0
    dt_eff: float = 0.0
    n_unit: tuple = field(default_factory=tuple)
    profile: dict = field(default_factory=dict)

    def __post_init__(self):
        self.lnx = self.lny = self.lnz = self.lengthscale
        nf = int(math.ceil(self.fwidth * self.lengthscale))
        self.nfx = self.nfy = self.nfz = nf
        if self.ln_prf is not None:
            self.lnx = self.lny = self.lnz = self.ln_prf
        n1 = np.asarray(self.normal, dtype=np.float64)
        nrm = np.sqrt(n1[0] ** 2 + n1[1] ** 2 + n1[2] ** 2)
        self.n_unit = (n1[0] / nrm, n1[1] / nrm, n1[2] / nrm)
        V = W = 0
        if self.prf is None and self.profile1d is not None:
            self.profile = {k: np.array(self.profile1d[k], dtype=np.float64) for k in ("U", "uu", "vv", "ww", "uw")}
            U = self.profile["U"]
        elif self.prf is None:
            U, uu, vv, ww, uw = build_profile(self.mean_profile, "top-hat",
                                              self.bulk_velocity, self.u_dash, self.kma)
            self.profile = dict(U=U, uu=uu, vv=vv, ww=ww, uw=uw)
        else:
            self.profile = dict(self.prf)
            U, V, W = self.prf["U"], self.prf["V"], self.prf["W"]
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
                arr[arr < 0.0] = 0.0

    @property
    def P(self):
        return self.jma * self.kma

    @property
    def plane_shape(self):
        return (2 * self.nfy + self.jma, 2 * self.nfz + self.kma)

    @property
    def S(self):
        a, b = self.plane_shape
        return a * b

    @property
    def rotated(self):
        """main() rotates only when no profile file was given (profilefile == 'none', :1476)."""
        return self.prf is None and self.profile1d is None


def stream_plane_offset(cfg, c, p):
    """Offset (in doubles) of random plane p of component c in the MT19937 draw stream
    (draw order of digitalfilters.py:1361-1366 then :1460-1467)."""
    NX = 2 * cfg.nfx + 1
    if p < NX:
        return (c * NX + p) * cfg.S
    return (3 * NX + 3 * (p - NX) + c) * cfg.S


def stream_length(cfg):
    """Doubles of the stream that influence A: initial fill + (ns-1) steps (the draws made
    after the final filter are consumed by the reference but never used)."""
    NX = 2 * cfg.nfx + 1
    return 3 * cfg.S * (NX + max(cfg.ns - 1, 0))


def draw_stream(cfg, n=None):
    """The reference's RNG draws, digitalfilters.py:1361-1366,1460-1467: legacy MT19937
    uniform(-sqrt3, sqrt3), seeded like np.random.seed(seed)."""
    rs = np.random.RandomState(cfg.seed)
    return rs.uniform(low=-SQRT3, high=SQRT3, size=stream_length(cfg) if n is None else n)


# ----------------------------------------------------------------------------------------
# generation (digitalfilters.py:1403-1495)
# ----------------------------------------------------------------------------------------
def lund_point_coeffs(cfg):
    """Per-point (9, P) Lund parameters exactly as adapt1d / adapt2prf evaluate them:
    rows a00,a10,a11,a20,a21,a22,U,V,W (V,W = 0 and unused for the 1-D form)."""
    J, K = cfg.jma, cfg.kma
    pr = cfg.profile
    if cfg.prf is None and cfg.mean_profile in PROFILES_2D:
        co, um = adapt2d_point_coeffs(cfg.mean_profile, cfg.inner_d, pr["U"], pr["uu"], pr["vv"], pr["ww"],
                                      pr["uw"], J, K)
        out = np.zeros((9, J, K))
        out[:6] = np.stack(co)
        out[6] = um
        return out.reshape(9, J * K)
    if cfg.prf is None:
        co = lund1d_coeffs(pr["uu"], pr["vv"], pr["ww"], pr["uw"])
        rows = [np.broadcast_to(np.asarray(c, dtype=np.float64), (K,)) for c in co]
        rows.append(np.asarray(pr["U"], dtype=np.float64))
        out = np.zeros((9, J, K))
        for r in range(7):
            out[r] = rows[r][None, :]
        return out.reshape(9, J * K)
    co = lundprf_coeffs(pr["uu"], pr["vv"], pr["ww"], pr["uv"], pr["uw"], pr["vw"])
    out = np.stack(list(co) + [pr["U"], pr["V"], pr["W"]]).astype(np.float64)
    return out.reshape(9, J * K)


def generate(cfg, loops=False, steps=None, stream=None):
    """Snapshot matrix A (3P, ns) before mean subtraction -- main() :1403-1477."""
    P = cfg.P
    NX = 2 * cfg.nfx + 1
    taps = _taps(cfg)
    ns = cfg.ns if steps is None else steps
    if stream is None:
        rs = np.random.RandomState(cfg.seed)
        draw = lambda shape: rs.uniform(low=-SQRT3, high=SQRT3, size=shape)
    else:
        pos = [0]

        def draw(shape):
            n = int(np.prod(shape))
            v = stream[pos[0]:pos[0] + n].reshape(shape)
            pos[0] += n
            return v
    Jp, Kp = cfg.plane_shape
    xs = [draw((NX, Jp, Kp)) for _ in range(3)]
    A = np.zeros((3 * P, ns), dtype=np.float64)
    cache = {}
    for i in range(ns):
        col = _step_column(cfg, xs, taps, loops, cache)
        if i + 1 < ns:  # the draws after the final filter never reach A
            xs = [np.roll(x, -1, axis=0) for x in xs]
            for x in xs:
                x[NX - 1] = draw((Jp, Kp))
        A[:, i] = col
    return A


def _taps(cfg):
    return calccoeff(cfg.nfx, cfg.lnx), calccoeff(cfg.nfy, cfg.lny), calccoeff(cfg.nfz, cfg.lnz)


def _step_column(cfg, xs, taps, loops, cache):
    """One pass of the step loop body (main() :1440-1477): filter the three components'
    plane windows, Lund transform (adapt1d / adapt2d / adapt2prf), snapshot column, rotation."""
    J, K, P = cfg.jma, cfg.kma, cfg.P
    bx, by, bz = taps
    pr = cfg.profile
    if loops:
        ys = [filter_block_scipy(x, bx, by, bz) for x in xs]
    else:
        ys = [filter_block(x, bx, by, bz) for x in xs]
    if cfg.prf is None and cfg.mean_profile in PROFILES_2D:   # main() :1447-1449
        if "c" not in cache:
            cache["c"] = adapt2d_point_coeffs(cfg.mean_profile, cfg.inner_d, pr["U"], pr["uu"], pr["vv"],
                                              pr["ww"], pr["uw"], J, K)
        u, v, w = apply_lund(ys[0], ys[1], ys[2], cache["c"][0], cache["c"][1])
    elif cfg.prf is None:
        if loops:
            adapt1d_loops(ys[0], ys[1], ys[2], pr["U"], pr["uu"], pr["vv"], pr["ww"], pr["uw"], J, K)
            u, v, w = ys
        else:
            if "c" not in cache:
                cache["c"] = [np.broadcast_to(c, (K,)) for c in
                              lund1d_coeffs(pr["uu"], pr["vv"], pr["ww"], pr["uw"])]
            u, v, w = apply_lund(ys[0], ys[1], ys[2], cache["c"], pr["U"])
    else:
        if "c" not in cache:
            cache["c"] = lundprf_coeffs(pr["uu"], pr["vv"], pr["ww"], pr["uv"], pr["uw"], pr["vw"])
        u, v, w = apply_lund(ys[0], ys[1], ys[2], cache["c"], pr["U"], pr["V"], pr["W"])
    col = np.empty(3 * P)
    col[0:P] = u.reshape(P)
    col[P:2 * P] = v.reshape(P)
    col[2 * P:3 * P] = w.reshape(P)
    if cfg.rotated:
        if "R" not in cache:
            cache["R"] = rotation_matrix(*cfg.n_unit)
        R = cache["R"]
        if loops or not np.array_equal(R, np.eye(3)):
            col = rotate_velocity(col, R)
    return col


JUMP_MIN = 1 << 26   # doubles: ~0.5 s of sequential draws, about one jump's cost


def generate_steps(cfg, steps, chunk=1 << 24, jump=False):
    """Columns A[:, i] for the listed steps only, at any size: the planes step i filters
    (planes i..i+2nfx of each component, stream_plane_offset) are cut out of ONE sequential
    pass over the reference's draw stream (drawn in chunks and discarded), so late steps of a
    4096-step run cost one pass over ~0.9 G doubles instead of the whole step loop.
    jump=True skips gaps longer than JUMP_MIN doubles with the MT19937 jump-ahead of
    oracle.mt_jump (pinned against sequential numpy draws) instead of drawing them: a step
    53 G doubles into BASELINE config 5's stream then costs seconds, not minutes.
    Returns {step: column (3P,)}, each equal to generate(cfg)[:, step]."""
    NX = 2 * cfg.nfx + 1
    S = cfg.S
    Jp, Kp = cfg.plane_shape
    want = {}
    for i in steps:
        for c in range(3):
            for p in range(i, i + NX):
                want[stream_plane_offset(cfg, c, p)] = None
    starts = sorted(want)
    rs = np.random.RandomState(cfg.seed)
    pos = 0
    k = 0
    buf = np.empty(0)
    buf0 = 0
    while k < len(starts):
        need_end = starts[k] + S
        if buf0 + len(buf) < need_end:  # extend the window: keep the tail from starts[k]
            keep = buf[max(starts[k] - buf0, 0):] if starts[k] < buf0 + len(buf) else np.empty(0)
            if starts[k] >= buf0 + len(buf):  # skip ahead (draw and discard, or jump)
                if jump and starts[k] - pos > JUMP_MIN:
                    from .mt_jump import stream_at
                    rs = stream_at(cfg.seed, starts[k])
                    pos = starts[k]
                while pos < starts[k]:
                    n = min(chunk, starts[k] - pos)
                    rs.uniform(low=-SQRT3, high=SQRT3, size=n)
                    pos += n
                keep_start = pos
            else:
                keep_start = max(starts[k], buf0)
            n = max(chunk, need_end - pos)
            new = rs.uniform(low=-SQRT3, high=SQRT3, size=n)
            buf = np.concatenate([keep, new])
            buf0 = keep_start
            pos += n
        o = starts[k] - buf0
        want[starts[k]] = buf[o:o + S].reshape(Jp, Kp).copy()
        k += 1
    taps = _taps(cfg)
    out = {}
    cache = {}
    for i in steps:
        xs = [np.stack([want[stream_plane_offset(cfg, c, p)] for p in range(i, i + NX)]) for c in range(3)]
        out[i] = _step_column(cfg, xs, taps, False, cache)
    return out


def mean_and_center(A):
    """main() :1492-1495 -- mean over snapshots (numpy pairwise), then A[:,j] -= mean."""
    mean_field = np.mean(A, 1)
    Ac = A - mean_field[:, None]
    return mean_field, Ac


# ----------------------------------------------------------------------------------------
# POD (PODFS.py:1294-1393)
# ----------------------------------------------------------------------------------------
def num_valid_modes(energy, ns, tol_CN=1.0e-15):
    """PODFS.py:1312-1317, literally."""
    n = 0
    while ((energy[n].real / energy[0].real > pow(tol_CN, 2.0)) and (n < ns - 2)
           and (energy[n].real > 0.0)):
        n += 1
        if (energy[n].real / energy[0].real > pow(tol_CN, 2.0)) and (energy[n].real > 0.0):
            n += 1
    return n


def sort_eigen(energy, T):
    """sort_eigenvalues, PODFS.py:1430-1447: NaN -> -1e10 (mode zeroed); sort by
    (value, index) descending; columns permuted from the .real copy."""
    ns = len(energy)
    es = np.zeros(ns)
    T = np.array(T, copy=True)
    for k in range(ns):
        if math.isnan(energy[k].real) or math.isnan(energy[k].imag):
            es[k] = -1.0e10
            T[:, k] = 0.0
        else:
            es[k] = energy[k].real
    order = sorted(zip(es, range(ns)), reverse=True)
    idx = np.array([o[1] for o in order])
    return np.array([o[0] for o in order]), T.real[:, idx]


def pod(Ac, ns, nm, tol_CN=1.0e-15):
    """PODFS.POD with correct_for_cell_volumes='false' (digitalfilters.py:1500 call)."""
    C = np.dot(Ac[:, 0:ns].T, Ac[:, 0:ns]) / ns                       # :1455
    energy, T = np.linalg.eig(C)                                       # :1309
    energy, T = sort_eigen(energy, T)                                  # :1310
    nv = num_valid_modes(energy, ns, tol_CN)
    nmt = nm if (0 <= nm <= nv) else nv                                # :1319
    T = np.array(T, dtype=np.float64)
    for j in range(nv):                                                # :1323-1325
        mag = sum(T[:, j].real * T[:, j].real) / ns
        T[:, j] = T[:, j] * np.sqrt(energy[j].real / mag)
    inv = np.diag(np.ones(nmt) / energy[0:nmt].real, 0)               # :1331
    spatial = np.dot(np.dot(Ac[:, 0:ns], T[:, 0:nmt].real), inv) / ns  # :1333
    return dict(C=C, energy=energy, T=T, num_valid=nv, nm=nmt, spatial=spatial)


def scale_temporal_modes(T, energy, nv, ns):
    """PODFS.py:1323-1325 for an arbitrary eigenvector matrix (builtin sequential sum)."""
    T = np.array(T, dtype=np.float64, copy=True)
    for j in range(nv):
        mag = sum(T[:, j] * T[:, j]) / ns
        T[:, j] = T[:, j] * np.sqrt(energy[j] / mag)
    return T


# ----------------------------------------------------------------------------------------
# Fourier-series compression (PODFS.py:1523-1659)
# ----------------------------------------------------------------------------------------
def time_axis(ns, dt):
    """PODFS.py:1540-1542."""
    time = np.linspace(0, (ns - 1) * dt * 1, ns)
    period = time[-1] + (time[1] - time[0])
    return time, period


def dft_reference(y, time, period):
    """The literal expression of PODFS.py:1564-1571 for one mode -> complex64 (ns,)."""
    ns = len(y)
    c = np.zeros(ns, dtype=np.complex64)
    for n in range(ns):
        k = n - ns // 2
        ctemp = y * np.exp(-1j * 2 * k * np.pi * time / period)
        c[n] = ctemp.sum() / ctemp.size
    return c


def dft_explicit(y, time, period):
    """The same values, restated as the GPU computes them:
      zi = (-2k)*pi ; theta_m = (zi*t_m) * (1/period)      (numpy complex mul/div of a real)
      (cos, sin) = glibc cexp(0 + i theta) (== numpy complex exp)
      re_m = y_m cos - 0 sin ; im_m = y_m sin + 0 cos       (complex * real-cast)
      c = cpairwise_sum(re, im) * (1/ns)  -> complex64."""
    ns = len(y)
    inv_p = 1.0 / period
    inv_n = 1.0 / ns
    c = np.zeros(ns, dtype=np.complex64)
    for n in range(ns):
        k = n - ns // 2
        zi = (-2.0 * k) * math.pi
        th = (zi * time) * inv_p
        e = np.exp(1j * th)
        re = y * e.real - 0.0 * e.imag
        im = y * e.imag + 0.0 * e.real
        sr, si = cpairwise_sum(re, im)
        c[n] = complex(sr * inv_n, si * inv_n)
    return c


def rank_and_count(c, et):
    """PODFS.py:1575-1593: order by (|c| f32, n) descending; count coefficients until the
    float64 running sum of |c| reaches float64(sum_f32 |c|)*et (numpy-1.x promotion)."""
    ns = len(c)
    cmod = np.abs(c)                                   # float32
    order = np.lexsort((np.arange(ns), cmod))[::-1].astype(np.int32)
    energy_sum = np.float64(np.sum(np.abs(c)))
    energy = 0.0
    count = 0
    target = energy_sum * et
    while energy < target:
        energy += np.float64(cmod[order[count]])
        count += 1
    return order, count


def fourier(T, ns, dt, nm, et, explicit=False, loops=False):
    """fourier_coefficients (PODFS.py:1523-1659) -> dict(c, c_ind, c_count, FC, period)."""
    time, period = time_axis(ns, dt)
    c = np.zeros((ns, nm), dtype=np.complex64)
    c_ind = np.zeros((nm, ns), dtype=np.int32)
    c_count = np.zeros(nm, dtype=np.int64)
    for i in range(nm):
        y = np.asarray(T[:, i], dtype=np.float64)
        c[:, i] = dft_explicit(y, time, period) if explicit else dft_reference(y, time, period)
        c_ind[i], c_count[i] = rank_and_count(c[:, i], et)
        if loops:  # plot-only reconstruction y2 (PODFS.py:1603-1612), kept for CPU timing
            for x in time:
                f = 0
                for n in range(c_count[i]):
                    k = c_ind[i, n] - ns // 2
                    f += c[c_ind[i, n], i] * np.exp(1j * 2 * k * np.pi * x / period)
    FC = fc_rows(c, c_ind, c_count, ns)
    return dict(c=c, c_ind=c_ind, c_count=c_count, FC=FC, period=period, time=time)


def fc_rows(c, c_ind, c_count, ns):
    """i_d.FC rows [k, Re, Im] (PODFS.py:1629-1639)."""
    rows = []
    for i in range(len(c_count)):
        for j in range(c_count[i]):
            n = c_ind[i, j]
            rows.append([n - ns // 2, c[n, i].real, c[n, i].imag])
    return np.array(rows, dtype=np.float64).reshape(-1, 3)


def podfs_dat_text(nm, period, c, c_ind, c_count, ns):
    """PODFS.dat exactly as PODFS.py:1646-1659 writes it."""
    s = [str(nm), "\n" + str(period)]
    for i in range(nm):
        s.append("\n" + str(i + 1) + "\t" + str(c_count[i]))
    for i in range(nm):
        for j in range(c_count[i]):
            n = c_ind[i, j]
            s.append("\n" + str(n - ns // 2) + "\t" + str(c[n, i].real) + "\t" + str(c[n, i].imag))
    return "".join(s)


def eigenvalues_text(num_valid, ns, energy):
    """POD.eigenvalues.dat (PODFS.py:1409-1427)."""
    cum = np.zeros(num_valid)
    cum[0] = energy[0].real
    for i in range(1, num_valid):
        cum[i] = cum[i - 1] + energy[i].real
    total = cum[num_valid - 1]
    out = ["#\n",
           "# mode, energy, cumulative, percenterage energy, percentage cumulative, condition number (absolute value if negative)\n",
           "#\t\tNote: cummulative energies are set to zero after first negative energy",
           "#\n"]
    for i in range(num_valid):
        out.append("%4.1d %18.10e %18.10e %18.10e %18.10e %18.10e\n" % (
            i + 1, energy[i].real, cum[i], energy[i].real / total * 100.0,
            cum[i] / total * 100.0, math.sqrt(energy[i].real / energy[0].real)))
    for i in range(num_valid, ns):
        out.append("%4.1d %18.10e %18.10e %18.10e %18.10e %18.10e\n" % (
            i + 1, energy[i].real, 0.0, energy[i].real / total * 100.0, 0.0,
            math.sqrt(abs(energy[i].real / energy[0].real))))
    return "".join(out)


# ----------------------------------------------------------------------------------------
# whole path
# ----------------------------------------------------------------------------------------
def run(cfg, loops=False):
    A = generate(cfg, loops=loops)
    mean_field, Ac = mean_and_center(A)
    res = pod(Ac, cfg.ns, cfg.nm)
    fo = fourier(res["T"], cfg.ns, cfg.dt_eff, res["nm"], cfg.et, loops=loops)
    res.update(A_raw=A, mean_field=mean_field, fourier=fo)
    return res
