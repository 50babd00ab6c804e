"""Host-side cost of one 64-document ingest batch (chunking, preprocess, encoder / decoder
tokenization) — the CPU work that precedes the GPU work of an ingest batch."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402
from docagents_amd.models.bert import pack_for_encoder  # noqa: E402
from docagents_amd.models.configs import decoder_config, encoder_config  # noqa: E402
from docagents_amd.models.tokenizer import decoder_tokenizer, encoder_tokenizer  # noqa: E402
from docagents_amd.text.chunker import Options, chunk_text  # noqa: E402
from docagents_amd.text.preprocess import preprocess_text  # noqa: E402

enc = encoder_tokenizer(encoder_config("bge-base").vocab)
dec = decoder_tokenizer(decoder_config("phi3-mini").vocab)
dg = B.TextGen(seed=500)
docs = [dg.document(2000) for _ in range(64)]
t = time.perf_counter()
chunks = []
for j, d in enumerate(docs):
    chunks.extend(f"Document: doc{j}.txt\n\n{c.text}" for c in chunk_text(d, Options(400, 80)))
t1 = time.perf_counter()
pp = [preprocess_text(c) for c in chunks]
t2 = time.perf_counter()
seqs = pack_for_encoder(enc, pp, 512, {"embed_truncated_texts": 0, "embed_truncated_tokens": 0})
t3 = time.perf_counter()
ids = [dec.encode(d, add_special_tokens=False).ids for d in docs]
t4 = time.perf_counter()
print(f"{len(chunks)} chunks: chunk {1e3 * (t1 - t):.1f} ms, preprocess {1e3 * (t2 - t1):.1f}, "
      f"encoder tokenize {1e3 * (t3 - t2):.1f}, decoder tokenize {1e3 * (t4 - t3):.1f} ms "
      f"({sum(map(len, ids)) / 64:.0f} decoder tokens / doc, {type(enc).__name__}, {type(dec).__name__})")
