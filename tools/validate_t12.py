import json, os, numpy as np, scipy.linalg as sl, mpmath as mp
C = {k: [float(v) for v in vals] for k, vals in json.load(open(os.path.join(os.environ.get('TMPDIR', '/tmp'), 'coeffs_t12.json'))).items()}
def t12(A):
    I = np.eye(A.shape[0]); A2 = A @ A; A3 = A2 @ A
    B = {k: c[0] * I + c[1] * A + c[2] * A2 + c[3] * A3 for k, c in C.items()}
    A6 = B['b3'] + B['b4'] @ B['b4']
    return B['b1'] + (B['b2'] + A6) @ A6
def ps14(A):
    f = [1 / np.math.factorial(k) if hasattr(np, 'math') else None for k in range(15)]
    import math
    f = [1 / math.factorial(k) for k in range(15)]
    I = np.eye(A.shape[0]); A2 = A @ A; A3 = A2 @ A
    Bi = lambda i: f[3 * i] * I + f[3 * i + 1] * A + f[3 * i + 2] * A2
    V = Bi(4)
    for i in range(3, -1, -1): V = A3 @ V + Bi(i)
    return V
def exact(A):
    M = mp.matrix(A.tolist()); E = mp.expm(M)
    return np.array(E.tolist(), dtype=complex)
mp.mp.dps = 30
rng = np.random.default_rng(1)
for N, th in [(40, 0.335), (40, 0.2), (27, 0.335), (9, 0.335), (9, 0.05)]:
    e12 = eps = 0
    for t in range(3):
        G = rng.normal(size=(N, N)) + 1j * rng.normal(size=(N, N)); H = (G + G.conj().T) / 2
        A = -1j * H; A *= th / np.abs(A).sum(0).max()
        X = exact(A)
        e12 = max(e12, np.abs(t12(A) - X).max()); eps = max(eps, np.abs(ps14(A) - X).max())
    print(N, th, "T12 err %.2e   PS14 err %.2e" % (e12, eps))
