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
(csrc/kernels/*: route byte) -- the host never touches the non-fraud rows.  Any other
rule set is compiled by ``device_program`` into a small postfix program
(csrc/include/ccfd_abi.h ``ccfd_rule_prog``) that the same epilogue interprets per row
(csrc/kernels/rules.h), so the GPU route byte, counters, amount histogram and fraud
hand-off list stay exact for configurable rules too.

Evaluation is IEEE float32 on both sides (numpy float32 here, explicit round-to-nearest
f32 ops on the GPU, no FMA contraction), so the host and the device agree bit for bit;
``log1p`` may differ by one ulp between libm and the device.  Rule files: one rule per
line, ``#`` comments (``RuleSet.load``; config key ``router.rules`` / env ROUTER_RULES).
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
_FUNCS = {"abs": np.abs, "log1p": np.log1p, "min": np.fmin, "max": np.fmax}   # fmin/fmax = device fminf/fmaxf


class RuleError(ValueError):
    pass


# device opcodes (csrc/include/ccfd_abi.h enum ccfd_rule_opcode)
OP_END, OP_VAR, OP_CONST = 0, 1, 2
OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_NEG, OP_ABS, OP_LOG1P, OP_MIN, OP_MAX = 3, 4, 5, 6, 7, 8, 9, 10, 11
OP_GT, OP_GE, OP_LT, OP_LE, OP_EQ, OP_NE, OP_AND, OP_OR, OP_NOT = 12, 13, 14, 15, 16, 17, 18, 19, 20
MAX_OPS, MAX_STACK = 48, 8
PROG_DTYPE = np.dtype([("op", "<i2"), ("arg", "<i2"), ("imm", "<f4")])
_BINOPS = {ast.Add: OP_ADD, ast.Sub: OP_SUB, ast.Mult: OP_MUL, ast.Div: OP_DIV}
_CMPOPS = {ast.Gt: OP_GT, ast.GtE: OP_GE, ast.Lt: OP_LT, ast.LtE: OP_LE, ast.Eq: OP_EQ, ast.NotEq: OP_NE}
_CALLS = {"abs": (OP_ABS, 1), "log1p": (OP_LOG1P, 1), "min": (OP_MIN, 2), "max": (OP_MAX, 2)}


@dataclass
class Rule:
    name: str
    expr: str
    route: Route
    code: object = None


class _Vectorise(ast.NodeTransformer):
    """Rewrite a rule expression to float32 numpy semantics identical to the device
    interpreter: every value is a float32 array (comparisons and and/or/not yield 1.0/0.0,
    operands are true when != 0), literals are float32, chained comparisons are
    conjunctions."""

    @staticmethod
    def _call(name, *args):
        return ast.Call(func=ast.Name(id=name, ctx=ast.Load()), args=list(args), keywords=[])

    def visit_Constant(self, node):
        return self._call("_c", node)

    def visit_BoolOp(self, node):
        self.generic_visit(node)
        op = ast.BitAnd() if isinstance(node.op, ast.And) else ast.BitOr()
        out = self._call("_t", node.values[0])
        for v in node.values[1:]:
            out = ast.BinOp(left=out, op=op, right=self._call("_t", v))
        return self._call("_b", out)

    def visit_UnaryOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Not):
            return self._call("_b", ast.UnaryOp(op=ast.Invert(), operand=self._call("_t", node.operand)))
        return node

    def visit_Compare(self, node):
        self.generic_visit(node)
        parts, left = [], node.left
        for op, right in zip(node.ops, node.comparators):
            parts.append(ast.Compare(left=left, ops=[op], comparators=[right]))
            left = right
        out = parts[0]
        for p in parts[1:]:
            out = ast.BinOp(left=out, op=ast.BitAnd(), right=p)
        return self._call("_b", out)


_ONE, _ZERO = np.float32(1), np.float32(0)
_HELPERS = {"_c": np.float32, "_t": lambda x: np.asarray(x) != 0,
            "_b": lambda m: np.where(m, _ONE, _ZERO)}


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

    @classmethod
    def from_config(cls, router_cfg) -> "RuleSet":
        """config.RouterConfig -> the deployed rule set: ``rules`` (file or inline text, with
        FRAUD_THRESHOLD bound to ``fraud_threshold``) or the reference threshold rule."""
        if getattr(router_cfg, "rules", ""):
            return cls.load(router_cfg.rules, {"FRAUD_THRESHOLD": float(router_cfg.fraud_threshold)})
        return cls.threshold(router_cfg.fraud_threshold)

    @classmethod
    def load(cls, spec: str, constants: Optional[Dict[str, float]] = None) -> "RuleSet":
        """``spec``: a rule file path, or the rule text itself (contains ``when``/``otherwise``)."""
        import os
        if os.path.exists(spec):
            with open(spec) as f:
                return cls.parse(f.read(), constants)
        if re.search(r"\b(when|otherwise|else)\b", spec, re.I):
            return cls.parse(spec.replace(";", "\n"), constants)
        raise RuleError(f"rules: {spec!r} is neither a file nor rule text")

    # ------------------------------------------------------------------ device program
    def device_program(self) -> bytes:
        """Compile to the kernels' postfix program (``ccfd_rule_prog``: 16-byte header +
        MAX_OPS x {i16 op, i16 arg, f32 imm}).  Raises RuleError when the rule set does not
        fit (more than MAX_OPS ops or a deeper stack than MAX_STACK)."""
        ops: List[tuple] = []
        depth = [0, 0]                                  # current, max

        def emit(op, arg=0, imm=0.0, dstack=0):
            ops.append((op, arg, imm))
            depth[0] += dstack
            depth[1] = max(depth[1], depth[0])

        def expr(node):
            if isinstance(node, ast.Expression):
                return expr(node.body)
            if isinstance(node, ast.Constant):
                if not isinstance(node.value, (int, float, bool)):
                    raise RuleError(f"constant {node.value!r} is not a number")
                return emit(OP_CONST, 0, float(node.value), +1)
            if isinstance(node, ast.Name):
                if node.id in self.constants:
                    return emit(OP_CONST, 0, float(self.constants[node.id]), +1)
                if node.id == "proba":
                    return emit(OP_VAR, 0, 0.0, +1)
                name = "Amount" if node.id == "amount" else node.id
                return emit(OP_VAR, 1 + FEATURE_NAMES.index(name), 0.0, +1)
            if isinstance(node, ast.UnaryOp):
                expr(node.operand)
                if isinstance(node.op, ast.UAdd):
                    return None
                return emit(OP_NOT if isinstance(node.op, ast.Not) else OP_NEG)
            if isinstance(node, ast.BinOp):
                expr(node.left)
                expr(node.right)
                return emit(_BINOPS[type(node.op)], dstack=-1)
            if isinstance(node, ast.BoolOp):
                op = OP_AND if isinstance(node.op, ast.And) else OP_OR
                expr(node.values[0])
                for v in node.values[1:]:
                    expr(v)
                    emit(op, dstack=-1)
                return None
            if isinstance(node, ast.Compare):
                left = node.left
                for i, (op, right) in enumerate(zip(node.ops, node.comparators)):
                    expr(left)
                    expr(right)
                    emit(_CMPOPS[type(op)], dstack=-1)
                    if i:
                        emit(OP_AND, dstack=-1)
                    left = right
                return None
            if isinstance(node, ast.Call):
                code, nargs = _CALLS[node.func.id]
                if len(node.args) != nargs:
                    raise RuleError(f"{node.func.id}() takes {nargs} argument(s) in rules")
                for a_ in node.args:
                    expr(a_)
                return emit(code, dstack=1 - nargs)
            raise RuleError(f"construct {type(node).__name__} cannot run on the device")

        for r in self.rules:
            expr(ast.parse(r.expr, mode="eval"))
            emit(OP_END, int(r.route), 0.0, -1)
        if len(ops) > MAX_OPS:
            raise RuleError(f"rule set needs {len(ops)} device ops (max {MAX_OPS})")
        if depth[1] > MAX_STACK:
            raise RuleError(f"rule set needs a stack of {depth[1]} (max {MAX_STACK})")
        prog = np.zeros(MAX_OPS, PROG_DTYPE)
        for i, (op, arg, imm) in enumerate(ops):
            prog[i] = (op, arg, np.float32(imm))
        head = np.array([len(ops), int(self.default), len(self.rules), depth[1]], np.int32)
        return head.tobytes() + prog.tobytes()

    def feature_vars(self) -> set:
        """Transaction columns the rules read (``amount`` reported as ``Amount``); empty when
        the rules only look at ``proba`` -- the only rule sets G32 / G20 (binned) rows can route."""
        out = set()
        for r in self.rules:
            for n in ast.walk(ast.parse(r.expr, mode="eval")):
                if isinstance(n, ast.Name) and n.id not in self.constants and n.id not in _FUNCS \
                        and n.id != "proba":
                    out.add("Amount" if n.id == "amount" else n.id)
        return out

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
        """Vectorised: returns uint8 routes (1 = fraud) for a batch (float32 arithmetic, the
        same as the device interpreter)."""
        proba = np.asarray(proba, np.float32).reshape(-1)
        n = proba.shape[0]
        env: Dict[str, object] = {k: np.float32(v) for k, v in self.constants.items()}
        env.update(_FUNCS)
        env.update(_HELPERS)
        env["proba"] = proba
        if X is not None:
            X = np.asarray(X)
            for j, name in enumerate(FEATURE_NAMES):
                env[name] = X[:, j].astype(np.float32)
            env["amount"] = env["Amount"]
        elif amount is not None:
            env["amount"] = env["Amount"] = np.asarray(amount, np.float32).reshape(-1)
        out = np.full(n, int(self.default), np.uint8)
        decided = np.zeros(n, bool)
        for r in self.rules:
            try:
                with np.errstate(all="ignore"):
                    m = eval(r.code, {"__builtins__": {}}, env) != 0   # noqa: S307 (whitelisted AST)
            except KeyError as e:
                raise RuleError(f"rule {r.name!r} needs {e} which this call did not provide") from None
            m = np.broadcast_to(np.asarray(m, bool), (n,)) & ~decided
            out[m] = int(r.route)
            decided |= m
        return out


def run_device_program(prog: bytes, proba: np.ndarray, X: np.ndarray) -> np.ndarray:
    """Host reference interpreter of a ``device_program`` (float32, like csrc/kernels/rules.h):
    uint8 routes for rows X [n, 30] with proba [n]."""
    head = np.frombuffer(prog, np.int32, 4)
    n_ops, default = int(head[0]), int(head[1])
    ops = np.frombuffer(prog, PROG_DTYPE, MAX_OPS, 16)[:n_ops]
    proba = np.asarray(proba, np.float32).reshape(-1)
    X = np.asarray(X, np.float32)
    n = proba.shape[0]
    one, zero = np.float32(1), np.float32(0)
    st: List[np.ndarray] = []
    decided = np.zeros(n, bool)
    fraud = np.full(n, default != 0)
    with np.errstate(all="ignore"):
        for op, arg, imm in ops.tolist():
            if op == OP_VAR:
                st.append(proba if arg == 0 else X[:, arg - 1])
            elif op == OP_CONST:
                st.append(np.full(n, np.float32(imm)))
            elif op == OP_END:
                cond = st.pop() != 0
                fraud = np.where(~decided & cond, arg != 0, fraud)
                decided |= cond
            elif op in (OP_NEG, OP_ABS, OP_LOG1P, OP_NOT):
                a = st.pop()
                st.append({OP_NEG: lambda: -a, OP_ABS: lambda: np.abs(a), OP_LOG1P: lambda: np.log1p(a),
                           OP_NOT: lambda: np.where(a == 0, one, zero)}[op]().astype(np.float32))
            else:
                b = st.pop()
                a = st.pop()
                r = {OP_ADD: lambda: a + b, OP_SUB: lambda: a - b, OP_MUL: lambda: a * b, OP_DIV: lambda: a / b,
                     OP_MIN: lambda: np.fmin(a, b), OP_MAX: lambda: np.fmax(a, b),
                     OP_GT: lambda: a > b, OP_GE: lambda: a >= b, OP_LT: lambda: a < b, OP_LE: lambda: a <= b,
                     OP_EQ: lambda: a == b, OP_NE: lambda: a != b,
                     OP_AND: lambda: (a != 0) & (b != 0), OP_OR: lambda: (a != 0) | (b != 0)}[op]()
                st.append(np.where(r, one, zero) if r.dtype == bool else r.astype(np.float32))
    return fraud.astype(np.uint8)


def _route(s: str) -> Route:
    s = s.lower()
    if s in ("fraud", "fraudulent"):
        return Route.FRAUD
    if s in ("standard", "normal", "legit"):
        return Route.STANDARD
    raise RuleError(f"unknown route {s!r}")
