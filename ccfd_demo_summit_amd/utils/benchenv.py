"""What a benchmark line must say about the environment it ran in.

Every ``CCFD_*`` / ``HIP_*`` / ``HSA_*`` / ``GPU_*`` / ``AMD_*`` / ``ROC*`` variable the process
sees is recorded in the line.  They fall in three groups:

* **diagnostic**: the number is not a valid headline (an A/B library, injected faults,
  per-launch synchronisation, a sanitizer build, the removed round-1..4 ablation switch);
  ``bench.py`` refuses to print a line while one is set unless ``--diagnostic`` labels it;
* **tuning**: documented engine knobs (docs/TUNING.md) -- valid, but recorded so the line
  says which operating point it measured;
* everything else is recorded as-is (e.g. ``HSA_ENABLE_IPC_MODE_LEGACY``).
"""
from __future__ import annotations

import os
from typing import Dict, List, Mapping, Optional

PREFIXES = ("CCFD_", "HIP_", "HSA_", "GPU_", "AMD_", "ROCR_", "ROCM_", "NCCL_", "RCCL_")

# set => the measured work is not the production work, or the timing is distorted
DIAGNOSTIC = {
    "CCFD_ABLATE": "removed diagnostic ablation switch (round 1-4); never valid in a headline",
    "CCFD_LIB_PATH": "loads an A/B build of the native library (scripts/build_ab.py)",
    "CCFD_FAULTS": "fault injection (utils/faults.py): delays / stalls / crashes a rank",
    "CCFD_DEBUG_SYNC": "synchronises after every launch (debug mode)",
    "CCFD_SYNC_ZC_ROWS": "synchronous zero-copy row debug path",
    "CCFD_STAMPER_DEBUG": "consumer stamper debug logging",
    "CCFD_SANITIZE": "sanitizer build of the host runtime",
    "HIP_LAUNCH_BLOCKING": "serialises every kernel launch",
    "AMD_SERIALIZE_KERNEL": "serialises every kernel launch",
    "AMD_SERIALIZE_COPY": "serialises every copy",
    "HSA_XNACK": "XNACK (page-fault retry) mode changes the code objects that run",
}

# documented operating-point knobs (docs/TUNING.md): valid, recorded
TUNING = {"CCFD_PERSIST_PIPE", "CCFD_PERSIST_ITEM_ROWS", "CCFD_MLP_WAVES", "CCFD_MLP_TPW", "CCFD_MLP_PF",
          "CCFD_MLP_REGW", "CCFD_MLP_WEIGHTS", "CCFD_GBDT_CPW", "CCFD_GBDT_R", "CCFD_GBDT_KERNEL",
          "CCFD_COHERENT_OUT", "CCFD_IDLE_FLUSH_US", "CCFD_COMPLETION_THREAD", "CCFD_KC_PARSE_THREADS",
          "CCFD_G32_INFLIGHT", "CCFD_G32_GLOBAL_LEAVES", "GPU_MAX_HW_QUEUES"}


def collect(environ: Optional[Mapping[str, str]] = None) -> Dict[str, str]:
    """Every runtime-relevant variable, sorted by name."""
    env = os.environ if environ is None else environ
    return {k: env[k] for k in sorted(env) if k.startswith(PREFIXES)}


def diagnostics(environ: Optional[Mapping[str, str]] = None) -> List[str]:
    """Names of the diagnostic variables that are set (non-empty, not "0")."""
    env = os.environ if environ is None else environ
    out = []
    for k in sorted(DIAGNOSTIC):
        v = env.get(k)
        if v is not None and v.strip() not in ("", "0"):
            out.append(k)
    return out


def describe(environ: Optional[Mapping[str, str]] = None) -> Dict[str, object]:
    """The line's ``env`` block: all recorded variables, and which of them are diagnostic /
    tuning."""
    rec = collect(environ)
    diag = diagnostics(environ)
    return {"vars": rec, "diagnostic": diag, "tuning": sorted(k for k in rec if k in TUNING)}


def refusal(environ: Optional[Mapping[str, str]] = None, allow: bool = False) -> Optional[str]:
    """The message bench.py exits with when a diagnostic variable is set and the run is not
    labelled ``--diagnostic``; None when the line may be printed."""
    diag = diagnostics(environ)
    if not diag or allow:
        return None
    why = "; ".join(f"{k}: {DIAGNOSTIC[k]}" for k in diag)
    return (f"refusing to print a headline number with diagnostic environment set ({why}). "
            "Unset it, or pass --diagnostic to print a line labelled diagnostic")
