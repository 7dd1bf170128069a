"""MI355X-native multimodal prompt-retrieval VQA hot path (drop-in for tossowski/
MultimodalPromptRetrieval's encode -> retrieve -> prompt -> T5-generate path).

Python host surfaces mirror the reference (``T5VisionModel``, ``VQARetrieval`` with
``create_retrieval_dataset`` / ``retrieve_closest_qa_pairs``, ``utils.cosine_similarity``); the
arithmetic runs in ``libmpr.so`` (hand-written gfx950 HIP kernels, C ABI in include/mpr.h).
"""
# (``synthetic`` — seeded weights and inputs for tests and the bench — is not part of the API)
__all__ = ["dataset", "encoders", "index", "model", "t5", "tokenization", "utils"]
