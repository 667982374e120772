"""ccfd_demo_summit_amd -- MI355X-native streaming credit-card-fraud scoring framework.

Capabilities of ``ruivieira/ccfd-demo-summit`` (Kafka -> router -> Seldon model -> KIE
fraud process -> customer notification loop, Prometheus/Grafana), re-designed around
a GPU-resident micro-batcher and hand-written CDNA4 (gfx950) HIP kernels.  See
SURVEY.md for the reference analysis and README.md for the architecture.
"""
__version__ = "0.1.0"
