"""Operator analogue: the FraudDetection custom resource, its
rendering into Kubernetes manifests, and a local reconcile loop for one node.

    python -m ccfd_demo_summit_amd.launch operator --cr deploy/cr/frauddetection-mi355x.yaml --render out.yaml
    python -m ccfd_demo_summit_amd.launch operator --cr deploy/cr/frauddetection-mi355x.yaml --local
"""
from .local import LocalOperator, local_commands
from .render import dump, render, validate
from .spec import API_VERSION, KIND, FraudDetectionSpec, SpecError, from_odh, load, parse

__all__ = ["LocalOperator", "local_commands", "dump", "render", "validate", "API_VERSION", "KIND",
           "FraudDetectionSpec", "SpecError", "from_odh", "load", "parse"]
