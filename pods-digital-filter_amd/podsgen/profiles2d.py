"""adapt2d's 2-D profiles (digitalfilters.py:233-485) as per-point Lund parameters.

The reference re-splines the 1-D profile and re-factors the Reynolds-stress tensor at
every point inside every step; nothing there depends on the step, so the host evaluates
it once per run (O(P) numpy/scipy, the same FITPACK calls) and the GPU applies the result
per step with the j-varying Lund table (mode 0: u = a00 xu + 0 xv + 0 xw + Umean, v and w
without a mean, :305-307 / :391-393 / :483-485).
"""
import numpy as np

from .host import PROFILES_2D, _adapt2d_lund  # noqa: F401  (PROFILES_2D re-exported)


def _scalar_squares(x):
    """x[j]**2 as the reference evaluates it on numpy float64 SCALARS (C pow), which is not
    always the array fast path (x*x); only J + K values, so evaluate them one by one."""
    return np.array([x[i] ** 2 for i in range(len(x))], dtype=np.float64)


def _double_tanh(prof, J, K):
    """:238-307 -- the k profile times its own spline resampled along j (geometric mean)."""
    from scipy import interpolate
    uin, uuin, vvin, wwin, uwin = prof
    zArray = np.linspace(-1., 1, K)
    zi = np.linspace(-1., 1, J)
    inj = [interpolate.splev(zi, interpolate.splrep(zArray, v, s=0), der=0) for v in prof]
    for v, src in zip(inj, prof):                       # :248-258
        v[0] = src[0]
        v[-1] = src[-1]
    uinj, uuinj, vvinj, wwinj, uwinj = inj
    for v in (uuinj, vvinj, wwinj):                     # :262-268
        v[v < 0.] = 0.0
    with np.errstate(invalid="ignore"):
        R00 = np.sqrt(uuin[None, :] * uuinj[:, None])
        R11 = np.sqrt(vvin[None, :] * vvinj[:, None])
        R22 = np.sqrt(wwin[None, :] * wwinj[:, None])
        R20 = np.sign(uwin[None, :] + uwinj[:, None]) * np.sqrt(np.abs(uwin[None, :] * uwinj[:, None]))
        Umean = np.sqrt(uin[None, :] * uinj[:, None])
    return Umean, R00, R11, R22, R20


def _radial(prof, J, K, mean_profile, inner_d):
    """:309-393 (circular) and :395-485 (ring) -- the profile splined over r in [r_lo, 1]."""
    from scipy import interpolate
    uin = prof[0]
    x = np.linspace(-1., 1., J)
    y = np.linspace(-1., 1., K)
    ring = mean_profile == "ring-hyperbolic-tangent"
    if not ring:
        ci = int(np.argmax(uin))
        zArray = np.linspace(0, 1, len(uin) - ci)
        tcks = [interpolate.splrep(zArray, v[ci:], s=0) for v in prof]
        r_lo, at_lo = 0.0, [v[ci] for v in prof]
    else:
        zArray = np.linspace(inner_d, 1., K)
        tcks = [interpolate.splrep(zArray, v, s=0) for v in prof]
        r_lo, at_lo = inner_d, [v[0] for v in prof]
    r = np.sqrt(_scalar_squares(x)[:, None] + _scalar_squares(y)[None, :])
    vals = []
    for i, (tck, v) in enumerate(zip(tcks, prof)):
        e = np.asarray(interpolate.splev(r.ravel(), tck, der=0), dtype=np.float64).reshape(J, K)
        e = np.where(r == r_lo, at_lo[i], e)            # "reset boundaries to avoid dodgy values"
        e = np.where(r == 1.0, v[-1], e)
        e = np.where(r > 1.0, 0.0, e)                    # outside the unit circle: zero
        if ring:
            e = np.where(r < inner_d, 0.0, e)            # inside the inner ring: zero
        vals.append(e)
    return tuple(vals)


def adapt2d_factor(mean_profile, inner_d, uin, uuin, vvin, wwin, uwin, jma, kma):
    """Returns (a00, a10, a11, a20, a21, a22, Umean), each (jma, kma) float64."""
    J, K = int(jma), int(kma)
    prof = [np.array(np.broadcast_to(np.asarray(v, dtype=np.float64), (K,)))
            for v in (uin, uuin, vvin, wwin, uwin)]
    if mean_profile == "double-hyperbolic-tangent":
        Umean, R00, R11, R22, R20 = _double_tanh(prof, J, K)
    elif mean_profile in ("circular-hyperbolic-tangent", "ring-hyperbolic-tangent"):
        Umean, R00, R11, R22, R20 = _radial(prof, J, K, mean_profile, inner_d)
    else:
        raise ValueError("adapt2d: unknown mean_profile %r" % (mean_profile,))
    return _adapt2d_lund(R00, R11, R22, R20) + (Umean,)
