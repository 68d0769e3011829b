import sys, numpy as np
np.set_printoptions(linewidth=160, precision=5)
A = np.load(sys.argv[1]).astype(np.float64); B = np.load(sys.argv[2]).astype(np.float64)
ns = A.shape[0]
A = A.reshape(ns, 4, -1, 2); B = B.reshape(ns, 4, -1, 2)
mag = np.abs(A).reshape(ns, -1).max(axis=1)
e = np.abs(A - B) / mag[:, None, None, None]
print("max rel", e.max(), "bad subgrids", int((e.reshape(ns, -1).max(axis=1) > 1e-4).sum()))
print("per corr/reim max:", e.max(axis=(0, 2)))
s = int(np.argmax(e.reshape(ns, -1).max(axis=1)))
pix = np.where(e[s].max(axis=(0, 2)) > 1e-4)[0]
print("worst s", s, "bad pix", pix[:40])
for q in range(4):
    print(" corr", q, "A", A[s, q, pix[:3]].ravel(), "\n        B", B[s, q, pix[:3]].ravel())
