"""Dashboard conformance: do a Grafana dashboard's PromQL selectors match the series our
exporters serve?  (SURVEY.md §5 "reference dashboards load unchanged"; VERDICT r2 next #3.)

The reference ships six dashboards (deploy/grafana/*.json in the reference) whose panels
query the Seldon engine, the model container, the Camel router, KIE, Strimzi/JMX and Spark.
This module

* extracts every ``"expr"`` of a dashboard and the vector selectors in it
  (``name{label op "value", ...}``; aggregation clauses, functions, range selectors and
  numbers are skipped; Grafana template variables ``$x`` become ``.*``, their "All" value);
* scrapes Prometheus text exposition from endpoints, adding the target labels a Prometheus
  server would add (``instance`` = host:port, ``job``);
* reports every selector that matches no series.

    python -m ccfd_demo_summit_amd.metrics.promql DASHBOARD_DIR URL=JOB [URL=JOB ...]
"""
from __future__ import annotations

import json
import re
import sys
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

_FUNCS = {"sum", "rate", "irate", "round", "histogram_quantile", "count", "avg", "min", "max", "increase",
          "by", "without", "on", "ignoring", "group_left", "group_right", "and", "or", "unless", "offset",
          "abs", "delta", "deriv", "topk", "bottomk", "quantile", "stddev", "label_replace", "time", "vector",
          "scalar", "clamp_min", "clamp_max", "avg_over_time", "max_over_time", "min_over_time", "bool"}
_SEL = re.compile(r"([a-zA-Z_:][a-zA-Z0-9_:]*)\s*(\{[^}]*\})?")
_MATCH = re.compile(r'([a-zA-Z_][a-zA-Z0-9_]*)\s*(=~|!~|!=|=)\s*"((?:[^"\\]|\\.)*)"')


@dataclass
class Selector:
    name: str
    matchers: List[Tuple[str, str, str]] = field(default_factory=list)    # (label, op, value)
    expr: str = ""

    def __str__(self):
        m = ",".join(f'{k}{op}"{v}"' for k, op, v in self.matchers)
        return f"{self.name}{{{m}}}" if m else self.name


def selectors(expr: str) -> List[Selector]:
    """Vector selectors of one PromQL expression."""
    e = re.sub(r"\$\{?[a-zA-Z_][a-zA-Z0-9_]*\}?", ".*", expr)          # template variables: "All"
    e = re.sub(r"\[[^\]]*\]", "", e)                                   # range selectors
    e = re.sub(r"\b(by|without|on|ignoring)\s*\([^)]*\)", "", e)       # grouping label lists
    out = []
    for m in _SEL.finditer(e):
        name, body = m.group(1), m.group(2)
        end = m.end()
        rest = e[end:].lstrip()
        if name in _FUNCS and (rest.startswith("(") or not body):
            continue
        if re.fullmatch(r"\d+(\.\d+)?(e[+-]?\d+)?", name, re.I) or (rest.startswith("(") and not body):
            continue
        prev = e[:m.start()].rstrip()
        if prev.endswith(("{", ",")) and "=" in rest[:3]:                # a label name inside {...}
            continue
        ms = [(k, op, v) for k, op, v in _MATCH.findall(body or "")]
        out.append(Selector(name, ms, expr))
    return out


def dashboard_exprs(doc) -> List[str]:
    """Every ``expr`` string of a Grafana dashboard (any nesting: rows, panels, targets)."""
    out: List[str] = []

    def walk(o):
        if isinstance(o, dict):
            for k, v in o.items():
                if k == "expr" and isinstance(v, str) and v.strip():
                    out.append(v)
                else:
                    walk(v)
        elif isinstance(o, list):
            for x in o:
                walk(x)
    walk(doc)
    return out


Series = Tuple[str, Dict[str, str]]


def parse_exposition(text: str, target_labels: Optional[Dict[str, str]] = None) -> List[Series]:
    from prometheus_client.parser import text_string_to_metric_families
    out: List[Series] = []
    for fam in text_string_to_metric_families(text):
        for s in fam.samples:
            lab = dict(s.labels)
            for k, v in (target_labels or {}).items():
                lab.setdefault(k, v)
            out.append((s.name, lab))
    return out


def scrape(url: str, job: str, timeout: float = 10.0, instance: Optional[str] = None) -> List[Series]:
    """GET a /metrics-style endpoint; add instance=host:port and job as Prometheus would
    (``instance`` overrides the address, as a relabel rule would)."""
    import urllib.request
    from urllib.parse import urlparse
    with urllib.request.urlopen(url, timeout=timeout) as r:
        text = r.read().decode()
    u = urlparse(url)
    return parse_exposition(text, {"instance": instance or f"{u.hostname}:{u.port}", "job": job})


def _ok(label_value: str, op: str, v: str) -> bool:
    if op == "=":
        return label_value == v
    if op == "!=":
        return label_value != v
    full = re.fullmatch(v, label_value) is not None
    return full if op == "=~" else not full


def matches(sel: Selector, series: Iterable[Series]) -> int:
    n = 0
    for name, lab in series:
        if name != sel.name:
            continue
        if all(_ok(lab.get(k, ""), op, v) for k, op, v in sel.matchers):
            n += 1
    return n


def check(exprs_by_source: Dict[str, Sequence[str]], series: Sequence[Series]) -> Dict:
    """{source: [expr, ...]} -> report: total selectors, matched, and the unmatched ones."""
    rep = {"selectors": 0, "matched": 0, "unmatched": [], "by_source": {}}
    for src, exprs in exprs_by_source.items():
        tot = ok = 0
        for ex in exprs:
            for sel in selectors(ex):
                tot += 1
                n = matches(sel, series)
                if n:
                    ok += 1
                else:
                    rep["unmatched"].append({"source": src, "selector": str(sel), "expr": ex})
        rep["by_source"][src] = {"selectors": tot, "matched": ok}
        rep["selectors"] += tot
        rep["matched"] += ok
    return rep


def main(argv=None):
    import glob
    import os
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        raise SystemExit(__doc__)
    exprs = {}
    for p in sorted(glob.glob(os.path.join(argv[0], "*.json"))):
        with open(p) as f:
            exprs[os.path.basename(p)] = dashboard_exprs(json.load(f))
    series: List[Series] = []
    for t in argv[1:]:
        url, _, job = t.partition("=")
        series += scrape(url, job or "ccfd")
    rep = check(exprs, series)
    print(json.dumps(rep, indent=1))
    return 0 if not rep["unmatched"] else 1


if __name__ == "__main__":
    sys.exit(main())
