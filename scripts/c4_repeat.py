"""C4 invariance check repeated in one process (flakiness probe): six segments as one batch vs one at a time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "fun-asr-gguf_amd")]
from fun_asr_gguf import create_asr_engine  # noqa: E402
from fun_asr_gguf.synthetic import synth_audio  # noqa: E402
from oracle import ctc as octc  # noqa: E402

SR = 16000
api = create_asr_engine("synthetic", "synthetic", "synthetic", "synthetic", verbose=False, model="full",
                        max_batch=6, n_ctx=512, n_predict=253, ignore_eos=True)
audio = synth_audio(300 * SR, 4000)
wins = octc.segments_info(300.0, 60.0, 4.0)
chunks = [audio[int(s * SR):int(e * SR)] for s, e in wins]
ones = [api.transcribe_batch([c], temperature=0.0)[0] for c in chunks]
bad = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    batch = api.transcribe_batch(chunks, temperature=0.0)
    diff = [b for b in range(6) if batch[b].text != ones[b].text or batch[b].aligned != ones[b].aligned]
    enc = api.models.engine.encode(chunks, want_enc=True, independent=True)
    encd = [b for b in range(6) if not (enc["audio_embd"][b] == api.models.engine.encode([chunks[b]])["audio_embd"][0]).all()]
    print(f"iter {it}: segments differing from one-at-a-time {diff}; independent-encode rows differing {encd}", flush=True)
    bad += bool(diff or encd)
api.cleanup()
sys.exit(1 if bad else 0)
