"""Routing rules compiled for the GPU epilogue (router/rules.py device_program ->
csrc/kernels/rules.h): the postfix program's host reference interpreter agrees with the
vectorised RuleSet.evaluate on random rule sets (both float32), limits are enforced, and
rule sets load from files / inline text / the ROUTER_RULES config key."""
import numpy as np
import pytest

from ccfd_demo_summit_amd.config import load_config
from ccfd_demo_summit_amd.data import generate
from ccfd_demo_summit_amd.router.rules import MAX_OPS, RuleError, RuleSet, run_device_program

RULES3 = """
when amount > 200 and proba >= 0.2 then fraud      # big-ticket, moderately suspicious
when V17 < -2.5 or abs(V14) > 4 then fraud
otherwise standard
"""


def _rand_expr(rng, depth=0):
    leaves = ["proba", "amount", "Time", "V1", "V4", "V10", "V12", "V14", "V17", "V28", "FRAUD_THRESHOLD"]
    r = rng.random()
    if depth > 2 or r < 0.3:
        return rng.choice(leaves) if rng.random() < 0.7 else f"{rng.normal() * 3:.4g}"
    if r < 0.45:
        return f"({_rand_expr(rng, depth + 1)} {rng.choice(['+', '-', '*', '/'])} {_rand_expr(rng, depth + 1)})"
    if r < 0.55:
        f = rng.choice(["abs", "log1p", "min", "max"])
        if f in ("min", "max"):
            return f"{f}({_rand_expr(rng, depth + 1)}, {_rand_expr(rng, depth + 1)})"
        return f"{f}({_rand_expr(rng, depth + 1)})"
    if r < 0.65:
        return f"-{_rand_expr(rng, depth + 1)}"
    return f"{_rand_expr(rng, depth + 1)} {rng.choice(['<', '<=', '>', '>=', '==', '!='])} {_rand_expr(rng, depth + 1)}"


def _rand_rule(rng):
    parts = [_rand_expr(rng) for _ in range(int(rng.integers(1, 3)))]
    cond = f" {rng.choice(['and', 'or'])} ".join(f"({p}) > 0" if rng.random() < 0.3 else p for p in parts)
    if rng.random() < 0.2:
        cond = f"not ({cond})"
    if rng.random() < 0.15:
        cond = f"-1 < {rng.choice(['V1', 'V2', 'proba'])} < 0.5"
    return cond


def test_three_rule_set_program_matches_evaluate():
    X, _ = generate(200_000, seed=7)
    p = np.random.default_rng(1).random(len(X)).astype(np.float32)
    rs = RuleSet.parse(RULES3)
    prog = rs.device_program()
    assert len(prog) == 16 + 8 * MAX_OPS
    a, b = rs.evaluate(p, X=X), run_device_program(prog, p, X)
    np.testing.assert_array_equal(a, b)
    assert 0 < a.sum() < len(a)


def test_random_rule_sets_agree():
    X, _ = generate(20_000, seed=8)
    p = np.random.default_rng(2).random(len(X)).astype(np.float32)
    rng = np.random.default_rng(3)
    checked = 0
    for _ in range(150):
        lines = [f"when {_rand_rule(rng)} then {rng.choice(['fraud', 'standard'])}" for _ in range(int(rng.integers(1, 4)))]
        lines.append(f"otherwise {rng.choice(['fraud', 'standard'])}")
        rs = RuleSet.parse("\n".join(lines), {"FRAUD_THRESHOLD": 0.5})
        try:
            prog = rs.device_program()
        except RuleError:
            continue                                   # too deep / too long for the device
        with np.errstate(all="ignore"):
            a = rs.evaluate(p, X=X)
        b = run_device_program(prog, p, X)
        np.testing.assert_array_equal(a, b, err_msg="\n".join(lines))
        checked += 1
    assert checked > 100


def test_limits_and_threshold_detection():
    deep = "when " + "1 + (" * 9 + "proba" + ")" * 9 + " > 2 then fraud"     # right-nested: 10 deep
    with pytest.raises(RuleError, match="stack"):
        RuleSet.parse(deep).device_program()
    long = "when " + " + ".join(["proba"] * 30) + " > 1 then fraud"
    with pytest.raises(RuleError, match="ops"):
        RuleSet.parse(long).device_program()
    assert RuleSet.threshold(0.3).threshold_only == 0.3
    assert RuleSet.parse(RULES3).threshold_only is None


def test_rules_from_file_inline_and_config(tmp_path):
    f = tmp_path / "rules.drl"
    f.write_text(RULES3)
    assert RuleSet.load(str(f)).device_program() == RuleSet.parse(RULES3).device_program()
    inline = RuleSet.load("when proba >= FRAUD_THRESHOLD then fraud; otherwise standard", {"FRAUD_THRESHOLD": 0.7})
    assert inline.threshold_only == 0.7
    cfg = load_config(None, environ={"ROUTER_RULES": str(f), "FRAUD_THRESHOLD": "0.4"})
    rs = RuleSet.from_config(cfg.router)
    assert len(rs.rules) == 2 and rs.threshold_only is None
    cfg = load_config(None, environ={"FRAUD_THRESHOLD": "0.4"})
    assert RuleSet.from_config(cfg.router).threshold_only == pytest.approx(0.4)
    with pytest.raises(RuleError):
        RuleSet.load("no such file and no rules")
