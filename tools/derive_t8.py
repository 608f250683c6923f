# Derivation of a 3-product evaluation of the degree-8 Taylor polynomial (the scheme of Bader, Blanes & Casas 2019
# for m = 8), coefficients re-derived here:
#   A2 = A A,  A4 = A2 (x1 A + x2 A2),  A8 = (x3 A2 + A4)(x4 I + x5 A + x6 A2 + x7 A4),
#   T8 = I + A + y2 A2 + A8 = sum_{k <= 8} A^k / k!  exactly.
# Matching degrees 3..8 of A8 to 1/k! with the gauge x7 = 1 leaves a quadratic in x3; both roots (and both signs
# of x2) are exact schemes, the one with the smallest rounding-growth proxy at ||A|| = theta is kept.
# Offline tool (mpmath); prints the coefficients and the check against the Taylor coefficients.
import itertools

import mpmath as mp

mp.mp.dps = 60
F = [mp.mpf(1) / mp.factorial(k) for k in range(9)]


def schemes():
    out = []
    for sgn in (1, -1):
        x7 = mp.mpf(1)
        x2 = sgn * mp.sqrt(F[8] / x7)
        x1 = F[7] / (2 * x2 * x7)
        S = (F[6] - x1 ** 2 * x7) / (x2 * x7)  # x3 x7 + x6 = S  (x7 = 1)
        # deg5: x1 x3 x7 + x1 x6 + x2 x5 = F5  ->  x1 S + x2 x5 = F5
        x5 = (F[5] - x1 * S) / x2
        # deg3: x3 x5 + x1 x4 = F3 -> x4 = (F3 - x3 x5) / x1 ; deg4: x3 x6 + x1 x5 + x2 x4 = F4, x6 = S - x3
        # -> x3 (S - x3) + x1 x5 + x2 (F3 - x3 x5) / x1 - F4 = 0
        a = -1
        b = S - x2 * x5 / x1
        c = x1 * x5 + x2 * F[3] / x1 - F[4]
        disc = b * b - 4 * a * c
        for r in (1, -1):
            x3 = (-b + r * mp.sqrt(disc)) / (2 * a)
            x6 = S - x3
            x4 = (F[3] - x3 * x5) / x1
            y2 = F[2] - x3 * x4
            out.append(dict(x=[x1, x2, x3, x4, x5, x6, x7], y2=y2))
    return out


def poly(x, y2):
    x1, x2, x3, x4, x5, x6, x7 = x
    L = [0, 0, x3, x1, x2, 0, 0, 0, 0]
    R = [x4, x5, x6, x7 * x1, x7 * x2, 0, 0, 0, 0]
    P = [mp.mpf(0)] * 9
    for i in range(9):
        for j in range(9 - i):
            P[i + j] += L[i] * R[j]
    P[0] += 1
    P[1] += 1
    P[2] += y2
    return P


def proxy(x, y2, th):
    x1, x2, x3, x4, x5, x6, x7 = x
    a2 = th ** 2
    a4 = a2 * (abs(x1) * th + abs(x2) * a2)
    L = abs(x3) * a2 + a4
    R = abs(x4) + abs(x5) * th + abs(x6) * a2 + abs(x7) * a4
    return a2 + a4 + L * R + 1 + th + abs(y2) * a2


if __name__ == "__main__":
    th = 0.648
    best = None
    for s in schemes():
        P = poly(s["x"], s["y2"])
        err = max(abs(P[k] - F[k]) for k in range(9))
        c = proxy(s["x"], s["y2"], th)
        print("err", mp.nstr(err, 5), "proxy", mp.nstr(c, 8), [mp.nstr(v, 20) for v in s["x"]], mp.nstr(s["y2"], 20))
        if err < 1e-50 and (best is None or c < best[0]):
            best = (c, s)
    print("chosen:")
    for k, v in enumerate(best[1]["x"], 1):
        print(f"  x{k} = {mp.nstr(v, 25)}")
    print(f"  y2 = {mp.nstr(best[1]['y2'], 25)}")
