"""Routing rules: the replacement for the Camel router's Drools rules (README.md:427; the
"Drools" box over the router in docs/diagram.png).

A rule set is an ordered list ``when <expr> then <route>`` with a final ``otherwise
<route>``; the first matching rule wins.  Expressions are a safe Python subset over
``proba`` (the model's proba_1), ``amount``, ``Time``, ``V1``..``V28`` and named
constants (``FRAUD_THRESHOLD`` ...), evaluated VECTORISED over a whole micro-batch::

    when proba >= FRAUD_THRESHOLD then fraud
    when amount > 10000 and proba >= 0.2 then fraud
    otherwise standard

The default rule set is exactly the reference's ``proba_1 >= FRAUD_THRESHOLD`` (deploy/
router.yaml:69-70).  When a rule set is that single threshold rule, ``threshold_only``
is set and the decision is taken inside the GPU scoring kernel's epilogue instead
(csrc/kernels/*: route byte) -- the host never touches the non-fraud rows.
"""
from __future__ import annotations

import ast
import re
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..contracts.outcomes import Route
from ..contracts.transaction import FEATURE_NAMES

_ALLOWED = (ast.Expression, ast.BoolOp, ast.And, ast.Or, ast.UnaryOp, ast.Not, ast.USub, ast.UAdd,
            ast.Compare, ast.Gt, ast.GtE, ast.Lt, ast.LtE, ast.Eq, ast.NotEq, ast.BinOp, ast.Add, ast.Sub,
            ast.Mult, ast.Div, ast.Name, ast.Load, ast.Constant, ast.Call)
_FUNCS = {"abs": np.abs, "log1p": np.log1p, "min": np.minimum, "max": np.maximum}


class RuleError(ValueError):
    pass


@dataclass
class Rule:
    name: str
    expr: str
    route: Route
    code: object = None


class _Vectorise(ast.NodeTransformer):
    """and/or/not -> & | ~ on boolean arrays; chained comparisons -> conjunction."""

    def visit_BoolOp(self, node):
        self.generic_visit(node)
        op = ast.BitAnd() if isinstance(node.op, ast.And) else ast.BitOr()
        out = node.values[0]
        for v in node.values[1:]:
            out = ast.BinOp(left=out, op=op, right=v)
        return out

    def visit_UnaryOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Not):
            return ast.UnaryOp(op=ast.Invert(), operand=node.operand)
        return node

    def visit_Compare(self, node):
        self.generic_visit(node)
        if len(node.ops) == 1:
            return node
        parts, left = [], node.left
        for op, right in zip(node.ops, node.comparators):
            parts.append(ast.Compare(left=left, ops=[op], comparators=[right]))
            left = right
        out = parts[0]
        for p in parts[1:]:
            out = ast.BinOp(left=out, op=ast.BitAnd(), right=p)
        return out


def _compile(expr: str, names: set):
    try:
        tree = ast.parse(expr, mode="eval")
    except SyntaxError as e:
        raise RuleError(f"bad rule expression {expr!r}: {e}") from None
    for n in ast.walk(tree):
        if not isinstance(n, _ALLOWED):
            raise RuleError(f"construct {type(n).__name__} not allowed in rule {expr!r}")
        if isinstance(n, ast.Name) and n.id not in names and n.id not in _FUNCS:
            raise RuleError(f"unknown name {n.id!r} in rule {expr!r}")
        if isinstance(n, ast.Call) and not (isinstance(n.func, ast.Name) and n.func.id in _FUNCS):
            raise RuleError(f"only {sorted(_FUNCS)} may be called in rules")
    tree = ast.fix_missing_locations(_Vectorise().visit(tree))
    return compile(tree, "<rule>", "eval")


_LINE = re.compile(r"^\s*(?:rule\s+\"(?P<name>[^\"]*)\"\s+)?when\s+(?P<expr>.+?)\s+then\s+(?P<route>\w+)\s*$", re.I)
_ELSE = re.compile(r"^\s*(?:otherwise|else)\s+(?P<route>\w+)\s*$", re.I)


class RuleSet:
    def __init__(self, rules: List[Rule], default: Route = Route.STANDARD, constants: Optional[Dict[str, float]] = None):
        self.constants = dict(constants or {})
        self.rules = rules
        self.default = default
        names = set(FEATURE_NAMES) | {"proba", "amount"} | set(self.constants)
        for r in self.rules:
            r.code = _compile(r.expr, names)

    @classmethod
    def threshold(cls, fraud_threshold: float = 0.5) -> "RuleSet":
        return cls.parse("when proba >= FRAUD_THRESHOLD then fraud\notherwise standard",
                         {"FRAUD_THRESHOLD": fraud_threshold})

    @classmethod
    def parse(cls, text: str, constants: Optional[Dict[str, float]] = None) -> "RuleSet":
        rules, default = [], Route.STANDARD
        for i, line in enumerate(text.splitlines()):
            line = line.split("#", 1)[0].strip()
            if not line:
                continue
            m = _LINE.match(line)
            if m:
                rules.append(Rule(m.group("name") or f"rule{i}", m.group("expr"), _route(m.group("route"))))
                continue
            m = _ELSE.match(line)
            if m:
                default = _route(m.group("route"))
                continue
            raise RuleError(f"line {i + 1}: cannot parse {line!r}")
        return cls(rules, default, constants)

    @property
    def threshold_only(self) -> Optional[float]:
        """The threshold if this rule set is exactly ``proba >= T -> fraud, else standard``."""
        if len(self.rules) != 1 or self.default != Route.STANDARD or self.rules[0].route != Route.FRAUD:
            return None
        e = self.rules[0].expr.replace(" ", "")
        if e == "proba>=FRAUD_THRESHOLD" and "FRAUD_THRESHOLD" in self.constants:
            return float(self.constants["FRAUD_THRESHOLD"])
        m = re.fullmatch(r"proba>=([0-9.eE+-]+)", e)
        return float(m.group(1)) if m else None

    def evaluate(self, proba: np.ndarray, X: Optional[np.ndarray] = None, amount: Optional[np.ndarray] = None) -> np.ndarray:
        """Vectorised: returns uint8 routes (1 = fraud) for a batch."""
        proba = np.asarray(proba, np.float64).reshape(-1)
        n = proba.shape[0]
        env: Dict[str, object] = dict(self.constants)
        env.update(_FUNCS)
        env["proba"] = proba
        if X is not None:
            X = np.asarray(X)
            for j, name in enumerate(FEATURE_NAMES):
                env[name] = X[:, j].astype(np.float64)
            env["amount"] = env["Amount"]
        elif amount is not None:
            env["amount"] = env["Amount"] = np.asarray(amount, np.float64).reshape(-1)
        out = np.full(n, int(self.default), np.uint8)
        decided = np.zeros(n, bool)
        for r in self.rules:
            try:
                m = eval(r.code, {"__builtins__": {}}, env)   # noqa: S307 (whitelisted AST)
            except KeyError as e:
                raise RuleError(f"rule {r.name!r} needs {e} which this call did not provide") from None
            m = np.broadcast_to(np.asarray(m, bool), (n,)) & ~decided
            out[m] = int(r.route)
            decided |= m
        return out


def _route(s: str) -> Route:
    s = s.lower()
    if s in ("fraud", "fraudulent"):
        return Route.FRAUD
    if s in ("standard", "normal", "legit"):
        return Route.STANDARD
    raise RuleError(f"unknown route {s!r}")
