"""Reference-compatible model package (mirrors the reference's wav2vec2/ package API)."""
