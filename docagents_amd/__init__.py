"""docagents_amd — an MI355X-native multi-agent RAG document system.

Capabilities of tomerlieber/doc-agents (gateway / parser / analysis / query agents over a task
queue, two cache layers, summary + RAG QA with confidence) with the outsourced compute
(OpenAI embeddings + chat, pgvector) replaced by on-node MI355X inference: hand-written gfx950 HIP
kernels (MFMA GEMMs, flash attention, RMSNorm/LayerNorm, RoPE, sampling, fused cosine top-k), an
in-HBM sharded vector index and RCCL collectives over xGMI.
"""
__version__ = "0.1.0"
