"""Prometheus metric names exported by the reference services.

Router (``ccd-fuse:8091/prometheus``, README.md:500-530).  Dots in the README names
become underscores and counters gain ``_total`` as in the dashboard queries
(deploy/grafana/Router.json:88,163,250,326).
KIE (``ccd-service:8090/rest/metrics``, README.md:509-514,532-537; KIE.json:91,255,419,581).
Model (``:8000/prometheus``, deploy/grafana/ModelPrediction.json:96,104,211,322).
Seldon engine histograms (deploy/grafana/SeldonCore.json:119,411,499-531).
"""

# ---- router -------------------------------------------------------------
TRANSACTION_INCOMING = "transaction_incoming"           # counter (README.md:524)
TRANSACTION_OUTGOING = "transaction_outgoing"           # counter{type} (README.md:525-526)
NOTIFICATIONS_OUTGOING = "notifications_outgoing"       # counter (README.md:527; Router.json:88)
NOTIFICATIONS_INCOMING = "notifications_incoming"       # counter{response} (README.md:528-530)

# ---- KIE ----------------------------------------------------------------
FRAUD_INVESTIGATION_AMOUNT = "fraud_investigation_amount"   # histogram (README.md:534)
FRAUD_APPROVED_LOW_AMOUNT = "fraud_approved_low_amount"     # histogram (README.md:535)
FRAUD_APPROVED_AMOUNT = "fraud_approved_amount"             # histogram (README.md:536)
FRAUD_REJECTED_AMOUNT = "fraud_rejected_amount"             # histogram (README.md:537)

# ---- model gauges (last request) ----------------------------------------
MODEL_GAUGES = ("proba_1", "Amount", "V17", "V10")

# ---- seldon engine ------------------------------------------------------
SELDON_SERVER_REQUESTS = "seldon_api_engine_server_requests_seconds"
SELDON_CLIENT_REQUESTS = "seldon_api_engine_client_requests_seconds"
SELDON_CLIENT_LABELS = ("status", "deployment_name", "predictor_name", "predictor_version",
                        "model_name", "model_image", "model_version")

# ---- new GPU engine metrics (not in the reference) ----------------------
GPU_PREFIX = "ccfd_gpu_"
GPU_BATCHES = GPU_PREFIX + "batches"                 # counter
GPU_ROWS = GPU_PREFIX + "rows"                       # counter
GPU_BATCH_LATENCY = GPU_PREFIX + "batch_latency_seconds"  # histogram
GPU_TX_PER_SEC = GPU_PREFIX + "tx_per_second"        # gauge
GPU_INFLIGHT = GPU_PREFIX + "inflight_batches"       # gauge
GPU_GLOBAL_FRAUD_RATE = GPU_PREFIX + "global_fraud_rate"  # gauge (all-reduced)
GPU_AMOUNT = GPU_PREFIX + "amount"                   # histogram{type} (device-side)

ROUTER_METRICS = (TRANSACTION_INCOMING, TRANSACTION_OUTGOING, NOTIFICATIONS_OUTGOING,
                  NOTIFICATIONS_INCOMING)
KIE_METRICS = (FRAUD_INVESTIGATION_AMOUNT, FRAUD_APPROVED_LOW_AMOUNT, FRAUD_APPROVED_AMOUNT,
               FRAUD_REJECTED_AMOUNT)

# Amount histogram bucket upper bounds shared by the KIE histograms and the device-side
# amount histogram kernel (csrc/kernels/common.h AMOUNT_BOUNDS must match).
AMOUNT_BUCKETS = (1.0, 5.0, 10.0, 25.0, 50.0, 100.0, 250.0, 500.0, 1000.0, 2500.0,
                  5000.0, 10000.0, 25000.0)
N_AMOUNT_BUCKETS = len(AMOUNT_BUCKETS) + 1   # + the +Inf bucket
