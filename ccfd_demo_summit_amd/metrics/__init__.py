from .exporter import (CONTENT_TYPE, GpuEngineCollector, KieMetrics, MetricsHub, ModelMetrics,
                       RouterMetrics)

__all__ = ["CONTENT_TYPE", "GpuEngineCollector", "KieMetrics", "MetricsHub", "ModelMetrics", "RouterMetrics"]
