"""CPU oracle for the encode -> retrieve -> prompt -> T5-generate hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker / the timed CPU baseline —
never as a product code path.  The product (``multimodalpromptretrieval_amd``) runs on the HIP
library ``libmpr.so`` and fails loudly when it is missing.

What it is: a plain restatement, in torch-CPU fp32 eager ops, of the reference's algorithms,
each function citing the reference file:line (or third-party algorithm) it follows:

* ``oracle.retrieval`` — dataset/VQAFeatureDataset.py:187-246 (cdist + argsort + vote/bucket
  prompt, all four return modes) and utils.py:57-62 (cosine_similarity).
* ``oracle.clip`` — openai CLIP ViT-B/32 ``encode_image`` and ``encode_text`` (third-party,
  unpinned git HEAD, README.md:14) and architectures/T5VisionModel.py:112-139
  (get_image_token_features).
* ``oracle.t5`` — transformers T5ForConditionalGeneration encoder / decoder / greedy generate
  (requirements.txt:9 pins transformers 4.26.1; the container has 5.15.0, same arithmetic).
* ``oracle.pipeline`` — architectures/T5VisionModel.py:141-216 (prepare_input / predict).

Pinning: ``tests/golden/make_goldens.py`` imports the reference itself in the build container
(with a stub ``clip`` module) and transformers' CLIP/T5 modules as the
second source for the third-party arithmetic, and commits the outputs as fixtures under
``tests/golden/``; ``tests/test_oracle_golden.py`` checks this package against them.
"""
