"""Data ingest for the hot path: Unreal HDR G-buffer screenshots (EXR per
channel) -> device content tensors, and the raw float32 tensor-buffer format. Mirrors
realtime_style_transfer/dataloaders/{common,hdrScreenshots,tensorbuffer}.py."""
