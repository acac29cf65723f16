"""paddle.incubate.optimizer.functional: BFGS and L-BFGS minimisation of a differentiable function of one
flat tensor, with a strong-Wolfe line search (reference python/paddle/incubate/optimizer/functional/
bfgs.py, lbfgs.py, line_search.py). The iteration runs on the tensors' device; the function value and its
gradient come from one autograd pass per evaluation."""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor, _wrap


def _eval(f, x):
    xx = x.detach().requires_grad_(True)
    with torch.enable_grad():
        v = f(_wrap(xx))
        vt = v._t if isinstance(v, Tensor) else v
        g, = torch.autograd.grad(vt.sum(), xx)
    return vt.detach().reshape(()), g.detach()


def _cubic_min(a0, f0, d0, a1, f1, d1):
    """Minimiser of the cubic through (a0, f0, d0), (a1, f1, d1), clamped into the interval."""
    d1_ = d0 + d1 - 3 * (f0 - f1) / (a0 - a1)
    disc = d1_ * d1_ - d0 * d1
    lo, hi = min(a0, a1), max(a0, a1)
    if disc >= 0:
        d2 = disc ** 0.5 * (1 if a1 > a0 else -1)
        t = a1 - (a1 - a0) * (d1 + d2 - d1_) / (d1 - d0 + 2 * d2)
        return min(max(t, lo), hi)
    return (lo + hi) / 2


def _strong_wolfe(f, x, fx, gx, p, a1=1.0, c1=1e-4, c2=0.9, max_iters=50):
    """Step length a with f(x + a p) <= f(x) + c1 a g.p and |g(x + a p).p| <= c2 |g.p| (Nocedal & Wright 3.5 /
    3.6, cubic interpolation in the zoom). Returns (a, f_new, g_new, evaluations)."""
    d0 = float((gx * p).sum())
    f0 = float(fx)
    a_prev, f_prev, d_prev = 0.0, f0, d0
    a = a1
    evals = 0
    fa = ga = None

    def zoom(lo, flo, dlo, hi, fhi, dhi):
        nonlocal evals
        for _ in range(max_iters):
            aj = _cubic_min(lo, flo, dlo, hi, fhi, dhi)
            if abs(aj - lo) < 1e-12 or abs(aj - hi) < 1e-12:
                aj = (lo + hi) / 2
            fj, gj = _eval(f, x + aj * p)
            evals += 1
            dj = float((gj * p).sum())
            if float(fj) > f0 + c1 * aj * d0 or float(fj) >= flo:
                hi, fhi, dhi = aj, float(fj), dj
            else:
                if abs(dj) <= -c2 * d0:
                    return aj, fj, gj
                if dj * (hi - lo) >= 0:
                    hi, fhi, dhi = lo, flo, dlo
                lo, flo, dlo = aj, float(fj), dj
            if abs(hi - lo) < 1e-14:
                break
        fj, gj = _eval(f, x + lo * p)
        evals += 1
        return lo, fj, gj

    for i in range(max_iters):
        fa, ga = _eval(f, x + a * p)
        evals += 1
        da = float((ga * p).sum())
        if float(fa) > f0 + c1 * a * d0 or (i > 0 and float(fa) >= f_prev):
            a, fa, ga = zoom(a_prev, f_prev, d_prev, a, float(fa), da)
            return a, fa, ga, evals
        if abs(da) <= -c2 * d0:
            return a, fa, ga, evals
        if da >= 0:
            a, fa, ga = zoom(a, float(fa), da, a_prev, f_prev, d_prev)
            return a, fa, ga, evals
        a_prev, f_prev, d_prev = a, float(fa), da
        a = a * 2.0
    return a, fa, ga, evals


def _prep(initial_position, dtype):
    x = initial_position._t if isinstance(initial_position, Tensor) else torch.as_tensor(initial_position)
    dt = {"float32": torch.float32, "float64": torch.float64}[str(dtype)]
    return x.detach().to(dt).reshape(-1).clone()


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7, tolerance_change=1e-9,
                  initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe", max_line_search_iters=50,
                  initial_step_length=1.0, dtype="float32", name=None):
    """Returns (is_converge, num_func_calls, position, objective_value, objective_gradient,
    inverse_hessian_estimate)."""
    if line_search_fn != "strong_wolfe":
        raise NotImplementedError("only line_search_fn='strong_wolfe' is supported")
    x = _prep(initial_position, dtype)
    n = x.numel()
    H = (initial_inverse_hessian_estimate._t.to(x.dtype).clone() if initial_inverse_hessian_estimate is not None
         else torch.eye(n, dtype=x.dtype, device=x.device))
    fx, g = _eval(objective_func, x)
    calls, done = 1, bool(g.abs().max() <= tolerance_grad)
    eye = torch.eye(n, dtype=x.dtype, device=x.device)
    for _ in range(max_iters):
        if done:
            break
        p = -(H @ g)
        a, f1, g1, ev = _strong_wolfe(objective_func, x, fx, g, p, initial_step_length,
                                      max_iters=max_line_search_iters)
        calls += ev
        s = a * p
        y = g1 - g
        x = x + s
        sy = float(s @ y)
        if sy > 1e-10:
            rho = 1.0 / sy
            V = eye - rho * torch.outer(s, y)
            H = V @ H @ V.t() + rho * torch.outer(s, s)
        change = abs(float(f1) - float(fx))
        fx, g = f1, g1
        if g.abs().max() <= tolerance_grad or change <= tolerance_change or s.abs().max() <= tolerance_change:
            done = True
    return done, calls, _wrap(x), _wrap(fx), _wrap(g), _wrap(H)


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50, tolerance_grad=1e-8,
                   tolerance_change=1e-8, initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe",
                   max_line_search_iters=50, initial_step_length=1.0, dtype="float32", name=None):
    """Returns (is_converge, num_func_calls, position, objective_value, objective_gradient). The search direction
    is the two-loop recursion over the last ``history_size`` (s, y) pairs."""
    if line_search_fn != "strong_wolfe":
        raise NotImplementedError("only line_search_fn='strong_wolfe' is supported")
    x = _prep(initial_position, dtype)
    H0 = initial_inverse_hessian_estimate._t.to(x.dtype) if initial_inverse_hessian_estimate is not None else None
    fx, g = _eval(objective_func, x)
    calls, done = 1, bool(g.abs().max() <= tolerance_grad)
    S, Y = [], []
    for _ in range(max_iters):
        if done:
            break
        q = g.clone()
        alphas = []
        for s, y in zip(reversed(S), reversed(Y)):
            r = 1.0 / float(y @ s)
            al = r * float(s @ q)
            q = q - al * y
            alphas.append((al, r))
        if H0 is not None:
            q = H0 @ q
        elif S:
            q = q * (float(S[-1] @ Y[-1]) / float(Y[-1] @ Y[-1]))
        for (al, r), s, y in zip(reversed(alphas), S, Y):
            b = r * float(y @ q)
            q = q + (al - b) * s
        p = -q
        a, f1, g1, ev = _strong_wolfe(objective_func, x, fx, g, p, initial_step_length,
                                      max_iters=max_line_search_iters)
        calls += ev
        s = a * p
        y = g1 - g
        x = x + s
        if float(s @ y) > 1e-10:
            S.append(s)
            Y.append(y)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
        change = abs(float(f1) - float(fx))
        fx, g = f1, g1
        if g.abs().max() <= tolerance_grad or change <= tolerance_change or s.abs().max() <= tolerance_change:
            done = True
    return done, calls, _wrap(x), _wrap(fx), _wrap(g)
