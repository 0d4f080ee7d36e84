"""fs2amd — MI355X-native FastSpeech2 mel-synthesis forward (HIP/CDNA4 kernels behind a C ABI)."""
