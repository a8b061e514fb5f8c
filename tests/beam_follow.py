"""Whole-window comparison of a decode run against the oracle's own arithmetic
(test infrastructure; used by tests/test_oracle_trace.py on CPU and
tests/test_gpu_beam_oracle.py on the device).

The guide is the oracle's token loop replayed on another producer's logits
(the device's, or on CPU a perturbed copy of the oracle's own): its decision
trace and the raw logits row of every prefix it decoded. The oracle then runs
on its OWN logits in follow mode (orc_trace_follow): at every traced decision
it takes the guide's outcome, and where its own arithmetic decided otherwise
the event comes back forced, with the oracle's distance to the guide's
outcome. So after a near-tie flip the comparison does not stop: every later
decision is again the oracle's arithmetic against the guide's, on the guide's
path. A logits tap pairs each row the oracle decodes with the guide's row for
the same (window, prefix), which gives the logits error exactly where each
decision was taken.

Bounds, with eps = max |guide - oracle| over the raw logits rows that fed the
window's decisions up to the step of the forced event (a log-prob moves by at
most 2 eps: logit + log-sum-exp):
  draw      cumulative-probability boundary of the taken id:   <= 2 eps
  argmax    top-1 - taken log-prob:                             <= 4 eps
  ts_mass   log sum p(ts) - max text lp:                        <= 4 eps
  assign    difference of two sums of n = step + 1 log-probs:   <= 4 eps n
  best      difference of two length-normalised scores:         <= 4 eps
  fallback / no_speech: avg log-prob or p(no speech) vs its threshold: <= 2 eps
and the check allows 2x each. At temperature t > 0 (fallback attempts) the
rules see logits / t, so eps / t takes eps's place. Structural events (decoder status, exact ties)
are never forced: a difference there ends following and fails the check.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

import orc


def noise_bound(ev: orc.TraceEv, eps: float) -> float:
    per = {"draw": 2 * eps, "argmax": 4 * eps, "ts_mass": 4 * eps,
           "assign": 4 * eps * (ev.step + 1), "best": 4 * eps, "fallback": 2 * eps,
           "no_speech": 2 * eps}
    return 2 * per.get(ev.kind, 0.0)  # structural kinds (status, exact_tie): 0


@dataclass
class FollowReport:
    decisions: int
    forced: List[Tuple[orc.TraceEv, float, float]]  # (event, distance, bound)
    eps_max: float
    rows: int
    tokens: List[int] = field(default_factory=list)
    kinds: Dict[str, int] = field(default_factory=dict)  # decisions checked per kind

    def summary(self, label: str) -> str:
        kinds: Dict[str, int] = {}
        for e, _, _ in self.forced:
            kinds[e.kind] = kinds.get(e.kind, 0) + 1
        worst = max((d / b for _, d, b in self.forced if b > 0), default=0.0)
        big = max(self.forced, key=lambda f: f[1], default=None)
        return (f"{label}: {self.decisions} decisions checked ({len(self.tokens)} tokens), "
                f"{len(self.forced)} forced near-tie flips {kinds or ''}; "
                f"largest flip distance {big[1]:.3g} ({big[0].kind}, bound {big[2]:.3g})"
                if big else
                f"{label}: {self.decisions} decisions checked ({len(self.tokens)} tokens), "
                f"0 forced flips")\
            + f"; max distance/bound {worst:.3f}; logits err max {self.eps_max:.3g} over "\
            f"{self.rows} rows"


def follow_compare(o: orc.Oracle, pcm, opt: orc.FullOptions, guide: List[orc.TraceEv],
                   guide_rows: Dict[Tuple[int, tuple], np.ndarray]) -> FollowReport:
    """Runs the oracle in follow mode against `guide` (its trace) and
    `guide_rows` ({(seek, prefix tokens): raw logits of the last position}),
    asserts every decision agrees or is a forced flip within the noise bound,
    and returns the report."""
    errs: Dict[Tuple[int, int], List[Tuple[int, float]]] = {}
    missing = []

    def tap(tokens, lg):
        seek, it, step, _ = orc.trace_ctx()
        ref = guide_rows.get((seek, tuple(tokens)))
        if ref is None:
            missing.append((seek, it, step, len(tokens)))
            return
        errs.setdefault((seek, it), []).append((step, float(np.abs(lg - ref).max())))

    (rc, segs, _, _), ta, brk = o.traced_follow(guide, pcm, opt, tap)
    assert rc == 0
    info = {"break": brk, "len": (len(ta), len(guide))}
    assert brk is None, (info, guide[brk] if brk < len(guide) else None,
                         ta[brk] if brk < len(ta) else None)
    assert [e.key() for e in ta] == [e.key() for e in guide], info
    assert not missing, missing[:4]  # the oracle decoded exactly the guide's prefixes
    assert not [e for e in ta if e.kind == "exact_tie"]  # D5 never decides here
    forced = []
    for i, e in enumerate(ta):
        if not e.forced:
            continue
        rows = errs[(e.seek, e.it)]
        # the rows decoded at trace step s feed the decisions of step s + 1
        eps = max(err for st, err in rows if st < e.step)
        t = opt.temperature + e.it * opt.temperature_inc
        if t > 0:
            eps /= t
        bound = noise_bound(e, eps)
        dist = e.fmargin
        g = guide[i]
        if e.kind == "draw":
            # same uniform on both sides; the boundary between the oracle's
            # own id and the taken id moved across it: its movement (>= the
            # oracle's distance) is what the logits noise must explain
            u = e.v
            assert g.v == u and g.lo <= u <= g.hi, (e, g)
            assert not (e.lo <= u < e.hi), e
            dist = abs(e.lo - g.lo) if e.own_b < e.b else abs(e.hi - g.hi)
            assert dist >= e.fmargin - 1e-12, (e, g)
        assert np.isfinite(dist) and dist <= bound, (i, e, g, eps, bound)
        forced.append((e, dist, bound))
    eps_max = max((err for rows in errs.values() for _, err in rows), default=0.0)
    toks = [t.id for s in segs for t in s.tokens]
    kinds: Dict[str, int] = {}
    for e in ta:
        kinds[e.kind] = kinds.get(e.kind, 0) + 1
    return FollowReport(len(ta), forced, eps_max, sum(len(r) for r in errs.values()), toks, kinds)
