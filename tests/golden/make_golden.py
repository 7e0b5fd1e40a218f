#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

This script is test infrastructure that runs ONLY in the build container, where the
reference tree is mounted read-only at /root/reference.  It imports the reference's own
``HMM/hmm_training.py`` / ``hmm_testing.py`` / ``hmm_classes.py`` (with empty stand-ins for
the feature-extraction libraries ``librosa``/``spectrum``/``seaborn`` that those modules import
at module scope but never call on the Baum-Welch path) and records, per case:

* the inputs (CSR symbols, N, M, epsilon, max_iterations, initial linear parameters);
* a per-iteration trace captured from the running ``hmm_training`` frame at the line right
  after the convergence scalar is computed (hmm_training.py:503-505): the convergence scalar
  L_k, the per-sequence log P(O|lambda_k), and the post-M-step unnormalised log-parameters;
* the returned (A, B, pi) (hmm_training.py:524-541) and the printed stdout lines;
* forward-only scores of every sequence under the returned model
  (hmm_testing.py:49-104, ``calculate_log_likelihood``).

Only the resulting ``.npz``/``.json`` data files travel; nothing here is imported by the
package, by the GPU tests or by bench.py.  Regenerate with:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import contextlib
import io
import json
import linecache
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    sys.dont_write_bytecode = True
    for name in ("librosa", "spectrum", "seaborn"):
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["spectrum"].poly2lsf = lambda *a, **k: None
    sys.modules["spectrum"].lsf2poly = lambda *a, **k: None
    sys.path.insert(0, os.path.join(REF, "HMM"))
    sys.path.insert(0, REF)
    import hmm_classes  # noqa: E402
    import hmm_testing  # noqa: E402
    import hmm_training  # noqa: E402

    # The trace hook keys on these reference lines; refuse to run against a different revision.
    src = hmm_training.__file__
    assert "current_log_likelihood_sum = log_sum_exp(log_probability_O_given_lambda)" in \
        linecache.getline(src, 503), "reference revision mismatch (line 503)"
    assert "if prev_log_likelihood_sum != float('-inf'):" in linecache.getline(src, 505)
    return hmm_training, hmm_testing, hmm_classes


HT, HTEST, HC = _import_reference()


# ----------------------------------------------------------------------------------------
# Input generators
# ----------------------------------------------------------------------------------------
def left_to_right(N: int, K: int):
    """The build's left-to-right generalisation of the reference's 4-state defaults
    (hmm_training.py:301-318): pi0=0.97 and 0.03/(N-1) elsewhere,
    a_ii=0.6, a_i,i+1=0.4, absorbing last state, B uniform."""
    pi = np.full(N, 0.03 / (N - 1)) if N > 1 else np.ones(1)
    pi[0] = 0.97 if N > 1 else 1.0
    A = np.zeros((N, N))
    for i in range(N - 1):
        A[i, i] = 0.6
        A[i, i + 1] = 0.4
    A[N - 1, N - 1] = 1.0
    B = np.full((N, K), 1.0 / K)
    return pi, A, B


def uniform_obs(rng, R, K, tlo, thi):
    return [rng.integers(0, K, size=int(rng.integers(tlo, thi + 1))).astype(np.int64) for _ in range(R)]


def hmm_obs(rng, R, N, K, tlo, thi, self_loop=0.9, conc=0.3):
    """Symbols sampled from a ground-truth left-to-right HMM with Dirichlet(conc) emissions:
    skewed symbol occupancy (SURVEY §8(d) distribution 'H')."""
    Bt = rng.dirichlet(np.full(K, conc), size=N)
    out = []
    for _ in range(R):
        T = int(rng.integers(tlo, thi + 1))
        s, seq = 0, []
        for _t in range(T):
            seq.append(rng.choice(K, p=Bt[s]))
            if s < N - 1 and rng.random() > self_loop:
                s += 1
        out.append(np.asarray(seq, dtype=np.int64))
    return out


# ----------------------------------------------------------------------------------------
# Running the reference with a trace hook
# ----------------------------------------------------------------------------------------
def run_reference(obs, N, M, epsilon, max_iterations, init=None, word="w"):
    """Call the reference hmm_training.  ``init`` = (pi, A, B) linear warm start written
    through the reference's own DataStorageHMM.save_hmm into ../Data/Eighty-five-percent_20
    relative to a scratch cwd (hmm_training.py:275-287); None = the reference defaults."""
    trace = []
    code = HT.hmm_training.__code__

    def local_tracer(frame, event, arg):
        if event == "line" and frame.f_lineno == 505:
            f = frame.f_locals
            trace.append(dict(
                iteration=int(f["iteration"]),
                L=float(f["current_log_likelihood_sum"]),
                logP=np.array(f["log_probability_O_given_lambda"], dtype=np.float64).copy(),
                log_pi=np.array(f["log_pi_matrix"], dtype=np.float64).copy(),
                log_A=np.array(f["log_a_matrix"], dtype=np.float64).copy(),
                log_B=np.array(f["log_b_matrix"], dtype=np.float64).copy(),
            ))
        return local_tracer

    def global_tracer(frame, event, arg):
        if event == "call" and frame.f_code is code:
            return local_tracer
        return None

    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "cwd"))
        if init is not None:
            pi0, A0, B0 = init
            model = HC.HMMTrained(N, M, np.asarray(A0), np.asarray(B0), np.asarray(pi0), word)
            HC.DataStorageHMM.save_hmm(model, base_dir=os.path.join(tmp, "Data", "Eighty-five-percent_20"),
                                       print_messages=False)
        os.chdir(os.path.join(tmp, "cwd"))
        buf = io.StringIO()
        try:
            sys.settrace(global_tracer)
            with contextlib.redirect_stdout(buf):
                A, B, pi = HT.hmm_training(obs, N=N, M=M, epsilon=epsilon, max_iterations=max_iterations,
                                           show_progress=True, word_name=word if init is not None else None,
                                           load_initial_params=init is not None)
        finally:
            sys.settrace(None)
            os.chdir(cwd)
    return A, B, pi, trace, buf.getvalue().splitlines()


def save_case(name, obs, N, M, epsilon, max_iterations, init, note):
    if init is None:
        pi0 = np.array([0.97, 0.02, 0.005, 0.005])
        A0 = np.array([[0.6, 0.4, 0.0, 0.0], [0.0, 0.6, 0.4, 0.0], [0.0, 0.0, 0.6, 0.4], [0.0, 0.0, 0.0, 1.0]])
        B0 = np.full((N, M), 1.0 / M)
        assert N == 4, "reference defaults are 4-state only (hmm_training.py:301-312)"
    else:
        pi0, A0, B0 = init
    A, B, pi, trace, lines = run_reference(obs, N, M, epsilon, max_iterations, init)
    model = HC.HMMTrained(N, M, A, B, pi, "w")
    scores = np.array([HTEST.calculate_log_likelihood(o, model) for o in obs if len(o) > 0])
    lengths = np.array([len(o) for o in obs], dtype=np.int64)
    offsets = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    symbols = np.concatenate(obs).astype(np.int64) if len(obs) else np.zeros(0, np.int64)
    it = len(trace)
    np.savez_compressed(
        os.path.join(OUT, f"bw_{name}.npz"),
        offsets=offsets, symbols=symbols, N=np.int64(N), M=np.int64(M),
        epsilon=np.float64(epsilon), max_iterations=np.int64(max_iterations),
        load_initial=np.bool_(init is not None),
        init_pi=np.asarray(pi0, np.float64), init_A=np.asarray(A0, np.float64), init_B=np.asarray(B0, np.float64),
        iterations=np.int64(it),
        trace_L=np.array([t["L"] for t in trace]),
        trace_logP=np.stack([t["logP"] for t in trace]) if it else np.zeros((0, len(obs))),
        trace_log_pi=np.stack([t["log_pi"] for t in trace]) if it else np.zeros((0, N)),
        trace_log_A=np.stack([t["log_A"] for t in trace]) if it else np.zeros((0, N, N)),
        trace_log_B=np.stack([t["log_B"] for t in trace]) if it else np.zeros((0, N, M)),
        out_A=A, out_B=B, out_pi=pi,
        score_loglik=scores,
        stdout=np.array(lines, dtype=str),
        note=np.array(note),
    )
    nz = int(np.sum(B == 0.0))
    print(f"[golden] {name}: N={N} M={M} R={len(obs)} sumT={lengths.sum()} iters={it} "
          f"L={trace[-1]['L'] if it else None:.6f} exact-zero B entries={nz} | {lines[-1]}")
    return A, B, pi, trace, lines


def main():
    os.makedirs(OUT, exist_ok=True)

    # 1. reference default 4-state init (hmm_training.py:299-320), small codebook.
    rng = np.random.default_rng(101)
    save_case("n4_k16_default", uniform_obs(rng, 5, 16, 20, 60), 4, 16, 1e-6, 3, None,
              "reference default init, uniform symbols, max_iterations stop")

    # 2. default init at K=256 as HMM/main.py train runs it (max_iterations=2, main.py:268).
    rng = np.random.default_rng(102)
    save_case("n4_k256_default", uniform_obs(rng, 6, 256, 30, 60), 4, 256, 1e-6, 2, None,
              "main.py train shape: N=4 default init, 2 iterations, many 1e-20 floors")

    # 3. cfg1 stand-in: N=5 via the warm-start path, T ~ U[40,120].
    rng = np.random.default_rng(1)
    save_case("n5_k256_cfg1", uniform_obs(rng, 4, 256, 40, 120), 5, 256, 1e-6, 2, left_to_right(5, 256),
              "cfg1 stand-in: N=5 warm start (left-to-right generalisation), 2 iterations")

    # 4. cfg2 stand-in: N=8, skewed (HMM-generated) symbols.
    rng = np.random.default_rng(2)
    save_case("n8_k256_cfg2", hmm_obs(rng, 5, 8, 256, 40, 120), 8, 256, 1e-6, 2, left_to_right(8, 256),
              "cfg2 stand-in: N=8 warm start, HMM-generated skewed symbols")

    # 5. cfg3 shape (T=200) on a few sequences.
    rng = np.random.default_rng(3)
    save_case("n8_k256_t200", uniform_obs(rng, 4, 256, 200, 200), 8, 256, 1e-6, 2, left_to_right(8, 256),
              "cfg3 shape T=200 N=8 K=256, R=4")

    # 6. a T=1 sequence (xi empty, dominates the convergence scalar: SURVEY Q2).
    rng = np.random.default_rng(106)
    obs = uniform_obs(rng, 4, 16, 10, 30)
    obs.insert(2, np.array([3], dtype=np.int64))
    save_case("t1_edge", obs, 4, 16, 1e-6, 3, None, "contains a T=1 sequence")

    # 7. convergence stop: search seeds for a run that converges before max_iterations.
    for seed in range(200, 260):
        rng = np.random.default_rng(seed)
        obs = uniform_obs(rng, 4, 8, 15, 15)
        A, B, pi, trace, lines = run_reference(obs, 4, 8, 1e-6, 100, None)
        if lines and lines[-1].startswith("Converged after") and len(trace) < 60:
            save_case("converge", obs, 4, 8, 1e-6, 100, None, f"convergence stop (seed {seed})")
            break
    else:
        raise RuntimeError("no converging seed found")

    # 8. B entries that safe_exp underflows to exactly 0.0.
    for seed in range(300, 400):
        rng = np.random.default_rng(seed)
        obs = uniform_obs(rng, 4, 12, 60, 120)
        A, B, pi, trace, lines = run_reference(obs, 4, 12, 1e-6, 3, None)
        if np.sum(B == 0.0) > 0:
            save_case("b_underflow", obs, 4, 12, 1e-6, 3, None, f"exact-zero B entries via safe_exp underflow (seed {seed})")
            break
    else:
        print("[golden] WARNING: no seed produced exact-zero B entries")

    # 9. unreachable state: empty A/B denominators leave rows at -inf (hmm_training.py:440,471).
    N, K = 4, 10
    pi0 = np.array([0.9, 0.1, 0.0, 0.0])
    A0 = np.array([[0.7, 0.3, 0, 0], [0, 1.0, 0, 0], [0, 0, 0.5, 0.5], [0, 0, 0, 1.0]])
    B0 = np.full((N, K), 1.0 / K)
    rng = np.random.default_rng(109)
    save_case("empty_rows", uniform_obs(rng, 4, K, 8, 20), N, K, 1e-6, 2, (pi0, A0, B0),
              "states 2,3 unreachable: empty denominators, pi zeros")

    # 10. zero-probability sequence (log P = -inf) still counts in R for pi.
    N, K = 4, 10
    pi0, A0, B0 = left_to_right(N, K)
    B0 = B0.copy()
    B0[:, 7] = 0.0
    B0 /= B0.sum(1, keepdims=True)
    rng = np.random.default_rng(110)
    obs = [o % 7 for o in uniform_obs(rng, 4, K, 10, 25)]
    obs[1] = obs[1].copy()
    obs[1][3] = 7
    save_case("zero_prob_seq", obs, N, K, 1e-6, 2, (pi0, A0, B0), "sequence 1 has probability 0 (log P=-inf)")

    # 11. dense (fully connected) transitions, N=6 (not a power of two).
    rng = np.random.default_rng(111)
    N, K = 6, 32
    pi0 = rng.dirichlet(np.ones(N))
    A0 = rng.dirichlet(np.ones(N), size=N)
    B0 = rng.dirichlet(np.ones(K), size=N)
    save_case("dense_n6", uniform_obs(rng, 5, K, 20, 50), N, K, 1e-6, 3, (pi0, A0, B0), "dense ergodic A, N=6")

    # 12. dense N=16 (16-lane groups).
    rng = np.random.default_rng(112)
    N, K = 16, 64
    pi0 = rng.dirichlet(np.ones(N))
    A0 = rng.dirichlet(np.ones(N) * 0.5, size=N)
    B0 = rng.dirichlet(np.ones(K), size=N)
    save_case("dense_n16", uniform_obs(rng, 3, K, 15, 30), N, K, 1e-6, 2, (pi0, A0, B0), "dense A, N=16")

    # 13. large-state shape (cfg5's N and K) at tiny R*T: left-to-right, N=64, K=1024, 1 iteration.
    rng = np.random.default_rng(5)
    save_case("n64_k1024_tiny", uniform_obs(rng, 2, 1024, 12, 16), 64, 1024, 1e-6, 1, left_to_right(64, 1024),
              "cfg5 state/codebook shape at tiny size, 1 iteration")

    # 14. get_observations (VQ, hmm_training.py:82-120): nearest centroid over mfcc[1:].
    rng = np.random.default_rng(114)
    K, D = 64, 13
    cents = rng.normal(size=(K, D))
    cents[5] = cents[9]  # duplicated centroid: first-min tie-break
    recs = [rng.normal(size=(int(rng.integers(5, 40)), D)) for _ in range(6)]
    recs[0][3] = cents[9]  # exact hit on the duplicated centroid
    ns = types.SimpleNamespace
    obs = HT.get_observations([[ns(mfcc=f) for f in r] for r in recs], [ns(mfcc=c) for c in cents])
    lengths = np.array([len(r) for r in recs], dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "vq_k64.npz"), centroids=cents,
                        frames=np.concatenate(recs), offsets=np.concatenate([[0], np.cumsum(lengths)]),
                        symbols=np.concatenate(obs).astype(np.int64))
    print(f"[golden] vq_k64: {len(recs)} recordings, {lengths.sum()} frames")

    # 15. the HMMTrained JSON schema as written by DataStorageHMM.save_hmm (hmm_classes.py:51-60).
    model = HC.HMMTrained(3, 4, np.array([[0.5, 0.5, 0.0], [0.0, 0.25, 0.75], [0.0, 0.0, 1.0]]),
                          np.array([[0.1, 0.2, 0.3, 0.4], [0.25, 0.25, 0.25, 0.25], [1e-20, 0.5, 0.5, 0.0]]),
                          np.array([0.97, 0.02, 0.01]), "golden")
    with tempfile.TemporaryDirectory() as tmp:
        HC.DataStorageHMM.save_hmm(model, base_dir=tmp, print_messages=False)
        with open(os.path.join(tmp, "golden.json")) as f:
            text = f.read()
    with open(os.path.join(OUT, "hmm_json_schema.json"), "w") as f:
        f.write(text)
    print("[golden] hmm_json_schema.json written")


if __name__ == "__main__":
    main()
