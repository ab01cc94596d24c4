"""oni355 -- an MI355X-native suspicious-connects engine with Open Network Insight's capabilities.

Layers: ingest/decoders (C++ ``liboni_native``), columnar day store, ML
(featurize → corpus → collapsed-Gibbs LDA → score; hand-written gfx950 kernels in
``liboni_hip`` + RCCL data parallelism), operational analytics (enrichment, feedback).
"""
__version__ = "0.1.0"
