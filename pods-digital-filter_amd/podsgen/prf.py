"""`.prf` inlet-profile reader (digitalfilters.py:524-1035).

Host-side setup, run once per job: a CFD code's plane of scattered points (x, y, z, u, v,
w and k with e or sdr, optionally uu/vv/ww) is rotated into the y-z plane, resampled on the
res-spaced (kma x jma) grid by scipy's linear `griddata`, rescaled to a mass flow or bulk
velocity, and turned into a per-point Reynolds-stress field by an eddy-viscosity model.
The result feeds adapt2prf (the per-point Lund table of the GPU generator, no rotation).

The arithmetic follows the reference line by line with the same numpy/scipy calls, so it
is bit-identical to it on the same numpy/scipy.  Python-2 semantics kept: `k**(3/2)` is
`k**1` (integer division, :758, :767, :779, :788).  The reference's nplotlib contour
plots of the fields (:851-872, :1011-1022) are not drawn (no VTK/matplotlib here; they do
not feed back into the results).
"""
import math

import numpy as np

_COLS = ("x", "y", "z", "u", "v", "w", "k", "e", "sdr", "uu", "vv", "ww")


def _header(profilefile):
    """:526-564 -- the `data,...` line: 0-based column of each named field (-1: absent)."""
    count = 0
    with open(profilefile, "r") as f:
        for line in f:
            count += 1
            if line.startswith("data"):
                names = line.strip().split(",")
                break
        else:
            raise ValueError("%s: no 'data' header line" % profilefile)
    cols = {c: -1 for c in _COLS}
    for i in range(1, len(names)):
        key = names[i].strip()
        if key in cols:
            cols[key] = i - 1
    return count, cols


def _axis_rotation(theta, nx, ny, nz):
    """Rotation by theta about (nx, ny, nz), the matrix of :649-651 / :669-671."""
    C = np.cos(theta)
    S = np.sin(theta)
    t = 1 - C
    return np.matrix([[t * nx ** 2 + C, t * nx * ny - S * nz, t * nx * nz + S * ny],
                      [t * nx * ny + S * nz, t * ny ** 2 + C, t * ny * nz - S * nx],
                      [t * nx * nz - S * ny, t * ny * nz + S * nx, t * nz ** 2 + C]])


def _rescale(U, V, W, k, eps, xn, yn, zn, scale_to, mdot_area_den=None):
    """:744-788 -- scale the velocities to a new mass flow (mdot_area_den = (A, den)) or
    bulk velocity, keeping the turbulence intensity and length scale of every point."""
    meanu, meanv, meanw = np.mean(U), np.mean(V), np.mean(W)
    udotn = meanu * xn + meanv * yn + meanw * zn
    flag = eps > 0
    TI = np.sqrt(2. / 3. * k[flag]) / np.sqrt(U[flag] ** 2 + V[flag] ** 2 + W[flag] ** 2)
    L = k[flag] ** 1 / eps[flag]                                  # Py2: 3/2 == 1
    if mdot_area_den is not None:
        A, den = mdot_area_den
        scale = scale_to / (udotn * A * den)
    else:
        scale = scale_to / udotn
    U, V, W = U * scale, V * scale, W * scale
    k[flag] = TI ** 2 * (U[flag] ** 2 + W[flag] ** 2 + V[flag] ** 2)
    eps[flag] = k[flag] ** 1 / L
    return U, V, W, k, eps


def read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad):
    """Returns (U, V, W, uu, vv, ww, uv, uw, vw) as (jma, kma) arrays, then lnx, kma, jma,
    the plane normal (xn, yn, zn) and centre (xc, yc, zc) -- the reference's tuple."""
    import warnings
    with warnings.catch_warnings():  # np.matrix, kept because the reference multiplies with it
        warnings.simplefilter("ignore", PendingDeprecationWarning)
        return _read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad)


def _read_prf(profilefile, res, mdot, den, bulk_velocity, non_dim, TestGrad):
    from scipy import interpolate
    count, col = _header(profilefile)
    try:                                                           # :566-569
        data = np.loadtxt(profilefile, skiprows=count)
    except Exception:
        data = np.loadtxt(profilefile, skiprows=count, delimiter=",")
    xA, yA, zA = data[:, col["x"]], data[:, col["y"]], data[:, col["z"]]
    UA, VA, WA = data[:, col["u"]], data[:, col["v"]], data[:, col["w"]]
    # in-plane vectors from the first two points and the first/last point (:596-602)
    x2, y2, z2 = xA[1] - xA[0], yA[1] - yA[0], zA[1] - zA[0]
    x1, y1, z1 = xA[-1] - xA[0], yA[-1] - yA[0], zA[-1] - zA[0]
    xn = y1 * z2 - z1 * y2                                         # :605-613
    yn = z1 * x2 - x1 * z2
    zn = x1 * y2 - y1 * x2
    nnorm = np.sqrt(xn ** 2 + yn ** 2 + zn ** 2)
    xn, yn, zn = xn / nnorm, yn / nnorm, zn / nnorm
    xc = (np.amax(xA) + np.amin(xA)) / 2                           # :616-618
    yc = (np.amax(yA) + np.amin(yA)) / 2
    zc = (np.amax(zA) + np.amin(zA)) / 2
    points = np.matrix([(xA - xc).T, (yA - yc).T, (zA - zc).T])  # :631-653
    points = _axis_rotation(-np.arccos(xn), 0, -zn, yn) * points   # normal onto x (:636-657)
    points = _axis_rotation(-np.arctan2(zn, yn), xn, yn, zn) * points  # twist (:638, :662-674)
    yspan = np.amax(points[1, :]) - np.amin(points[1, :])         # :677-680
    zspan = np.amax(points[2, :]) - np.amin(points[2, :])
    kma = int(math.ceil(zspan / res))
    jma = int(math.ceil(yspan / res))
    yArr, zArr = points[1, :], points[2, :]
    yi = np.linspace(np.min(yArr), np.min(yArr) + res * jma, jma)  # :695-700
    zi = np.linspace(np.min(zArr), np.min(zArr) + res * kma, kma)
    y, z = np.meshgrid(yi, zi)
    pts = points[1:, :].T

    def grid(vals, clamp):                                         # :712-739
        g = interpolate.griddata(pts, vals, (y, z), fill_value=0.0, method="linear")
        if clamp:
            g[g < 0] = 0
        return g
    U, V, W = grid(UA, False), grid(VA, False), grid(WA, False)
    k = grid(data[:, col["k"]], True) if col["k"] != -1 else None
    eps = grid(data[:, col["e"]], True) if col["e"] != -1 else None
    if col["sdr"] != -1:
        sdr = grid(data[:, col["sdr"]], True)
        eps = 0.09 * k * sdr                                       # :741-742
        eps[np.where(eps > 100000000)] = 0
    if mdot != 0.0:                                                # :745-768
        U, V, W, k, eps = _rescale(U, V, W, k, eps, xn, yn, zn, mdot, (res ** 2 * (kma - 1) * (jma - 1), den))
    elif bulk_velocity != 1.0:                                     # :770-788
        U, V, W, k, eps = _rescale(U, V, W, k, eps, xn, yn, zn, bulk_velocity)
    if TestGrad:                                                   # :795-798
        eps = np.ones(np.shape(U), dtype=np.float64)
        k = np.ones(np.shape(U), dtype=np.float64)
        k[0] = eps[0] = 0.0
    if k is None or eps is None:
        raise ValueError("%s: the eddy-viscosity model needs k and e (or sdr) columns" % profilefile)
    flag = np.where(eps == 0.0)                                    # :799-805
    flag1 = np.where(U == 0.0)
    U[flag] = 0
    V[flag] = 0
    W[flag] = 0
    k[flag] = 0
    eps[flag1] = 0
    if TestGrad:                                                   # :807-810
        U[:] = 1 * y + 2 * z
        V[:] = 3 * y + 4 * z
        W[:] = 5 * y + 6 * z
    dU, dV, dW = np.gradient(U, res), np.gradient(V, res), np.gradient(W, res)   # :812-828
    dUdy, dUdz, dVdy, dVdz, dWdy, dWdz = dU[1], dU[0], dV[1], dV[0], dW[1], dW[0]
    for g in (dUdy, dUdz, dVdy, dVdz, dWdy, dWdz):
        g[flag] = 0
    if not TestGrad:                                               # :831-845: 2x2 box means
        grads = [dUdy, dUdz, dVdy, dVdz, dWdy, dWdz]
        orig = [g.copy() for g in grads]
        for i in range(1, kma - 1):
            for j in range(1, jma - 1):
                for g, g1 in zip(grads, orig):
                    g[i, j] = np.mean(g1[i - 1:i + 1, j - 1:j + 1])
    if non_dim:                                                    # :847-849 (plots only)
        y = y / np.amax(z)
        z = z / np.amax(z)
    dUdx = -dVdy - dWdz                                            # :875
    dVdx = np.zeros((kma, jma), dtype=np.float64)                  # :880-881
    dWdx = np.zeros((kma, jma), dtype=np.float64)
    B = 2 * np.amax(points[1, :])                                  # :890-896
    Cw = 2 * np.amax(points[2, :])
    L = 0.07 * 2 * B * Cw / (B + Cw)
    lnx = math.ceil(L / res)
    nu_t = np.zeros((kma, jma), dtype=np.float64)                  # :996-1004
    f = np.where(eps > 0)
    nu_t[f] = 0.09 * k[f] ** 2 / eps[f]
    uu = -2. * nu_t * dUdx + 2. / 3. * k
    vv = -2. * nu_t * dVdy + 2. / 3. * k
    ww = -2. * nu_t * dWdz + 2. / 3. * k
    uv = -nu_t * (dUdy + dVdx)
    uw = -nu_t * (dUdz + dWdx)
    vw = -nu_t * (dVdz + dWdy)
    uu[np.where(uu < 0.0)] = 0.0                                   # :1007-1009
    vv[np.where(vv < 0.0)] = 0.0
    ww[np.where(ww < 0.0)] = 0.0
    out = [np.flip(a, 0).T for a in (U, V, W, uu, vv, ww, uv, uw, vw)]   # :1024-1035
    return tuple(out) + (lnx, kma, jma, xn, yn, zn, xc, yc, zc)
