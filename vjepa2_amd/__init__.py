"""vjepa2_amd — MI355X-native (gfx950) V-JEPA 2 pre-training step.

Host side mirrors the reference's module API (VisionTransformer / VisionTransformerPredictor /
MaskCollator / app.vjepa train step); the hot path runs in libvjepa_hip.so (include/vjepa_hip.h).
"""

__version__ = "0.1.0"
