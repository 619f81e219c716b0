"""Ghia, Ghia & Shin (1982) lid-driven cavity centreline data (published
reference data, as tabulated in the reference's
tests/validation/cavity_reference_data.h) and the RMS-error measure of
tests/validation/cavity_validation_utils.h:36-65,99-125."""
import math

Y = [0.0000, 0.0547, 0.0625, 0.0703, 0.1016, 0.1719, 0.2813, 0.4531, 0.5000, 0.6172, 0.7344,
     0.8516, 0.9531, 0.9609, 0.9688, 0.9766, 1.0000]
X = [0.0000, 0.0625, 0.0703, 0.0781, 0.0938, 0.1563, 0.2266, 0.2344, 0.5000, 0.8047, 0.8594,
     0.9063, 0.9453, 0.9531, 0.9609, 0.9688, 1.0000]
U = {
    100: [0.00000, -0.03717, -0.04192, -0.04775, -0.06434, -0.10150, -0.15662, -0.21090,
          -0.20581, -0.13641, 0.00332, 0.23151, 0.68717, 0.73722, 0.78871, 0.84123, 1.00000],
    1000: [0.00000, -0.18109, -0.20196, -0.22220, -0.29730, -0.38289, -0.27805, -0.10648,
           -0.06080, 0.05702, 0.18719, 0.33304, 0.46604, 0.51117, 0.57492, 0.65928, 1.00000],
}
V = {
    100: [0.00000, 0.09233, 0.10091, 0.10890, 0.12317, 0.16077, 0.17507, 0.17527, 0.05454,
          -0.24533, -0.22445, -0.16914, -0.10313, -0.08864, -0.07391, -0.05906, 0.00000],
    1000: [0.00000, 0.27485, 0.29012, 0.30353, 0.32627, 0.37095, 0.33075, 0.32235, 0.02526,
           -0.31966, -0.42665, -0.51550, -0.39188, -0.33714, -0.27669, -0.21388, 0.00000],
}


def interp(coords, vals, target):
    for i in range(len(coords) - 1):
        if coords[i] <= target <= coords[i + 1]:
            t = (target - coords[i]) / (coords[i + 1] - coords[i])
            return vals[i] + t * (vals[i + 1] - vals[i])
    return vals[-1]


def rms(coords, vals, ref_coords, ref_vals):
    s = 0.0
    for c, r in zip(ref_coords, ref_vals):
        e = interp(coords, vals, c) - r
        s += e * e
    return math.sqrt(s / len(ref_coords))


def centerlines(u2d, v2d, x, y):
    """u along x = x[nx/2] and v along y = y[ny/2] of a (ny, nx) plane."""
    ny, nx = u2d.shape
    ci, cj = nx // 2, ny // 2
    return list(y), [float(u2d[j, ci]) for j in range(ny)], list(x), \
        [float(v2d[cj, i]) for i in range(nx)]


def rms_errors(field, grid, re=100, k=0):
    y, uc, x, vc = centerlines(field.u[k], field.v[k], grid.x, grid.y)
    return rms(y, uc, Y, U[re]), rms(x, vc, X, V[re])


def rms_re100(field, grid):
    return rms_errors(field, grid, 100)
