"""The optimizer parity tolerance (north star: "BA pose deltas within 1e-5 relative").

The device sums the normal equations in trees, the oracle in the reference's sequential edge
order, so the two agree to rounding, not bit for bit. Both return f32 values. Per element:
  moved more than 1e-6 from the start value: |x - x_oracle| <= 1e-5 |x_oracle - x0| + 4 ulp
  otherwise:                                 |x - x_oracle| <= 1e-5 max |x_oracle - x0| + 4 ulp
with 4 ulp = 4 f32 epsilons of max(|x_oracle|, 1) (the f32 output rounding of either side)."""
import numpy as np

EPS32 = np.finfo(np.float32).eps
MOVED = 1e-6


def tolerance(A_ref, A0):
    A_ref, A0 = np.asarray(A_ref, np.float64), np.asarray(A0, np.float64)
    d = np.abs(A_ref - A0)
    dmax = d.max() if d.size else 0.0
    return np.where(d > MOVED, 1e-5 * d, 1e-5 * dmax) + 4 * EPS32 * np.maximum(np.abs(A_ref), 1.0)


def assert_close(A, A_ref, A0, what=""):
    A, A_ref = np.asarray(A, np.float64), np.asarray(A_ref, np.float64)
    tol = tolerance(A_ref, A0)
    err = np.abs(A - A_ref)
    bad = err > tol
    assert not bad.any(), (f"{what}: {int(bad.sum())} elements outside the tolerance; worst err "
                           f"{err[bad].max():.3g} vs tol {tol[bad][np.argmax(err[bad])]:.3g}")
