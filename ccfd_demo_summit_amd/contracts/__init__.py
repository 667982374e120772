"""Inter-service contracts: the API surface kept compatible with the reference demo.

The reference (`ruivieira/ccfd-demo-summit`) ships no source; its public surface is the
set of Kafka topics, env-var config keys, REST endpoints, Prometheus metric names and
business-process outcomes declared in its manifests.  Everything in
this framework imports those names from here, so there is exactly one source of truth.
"""
from .topics import Topics, DEFAULT_TOPICS
from .transaction import (
    FEATURE_NAMES, N_FEATURES, AMOUNT_COL, TIME_COL, Transaction,
    encode_tx_json, decode_tx_json, TxBatch,
    WIRE_ROW_BYTES, WIRE_PERM, encode_wire, decode_wire, G32_ROW_BYTES, encode_g32, amount_bucket,
    G20_ROW_BYTES, encode_g20, decode_g20_bins,
)
from .outcomes import Outcome, Route, CustomerResponse
from . import seldon, metric_names, env

__all__ = [
    "Topics", "DEFAULT_TOPICS", "FEATURE_NAMES", "N_FEATURES", "AMOUNT_COL", "TIME_COL",
    "Transaction", "encode_tx_json", "decode_tx_json", "TxBatch", "Outcome", "Route",
    "CustomerResponse", "seldon", "metric_names", "env",
]
