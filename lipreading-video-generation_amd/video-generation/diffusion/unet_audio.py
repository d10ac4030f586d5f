"""Drop-in for video-generation/diffusion/unet_audio.py on libvdiff (MI355X)."""
import _vdiff_path  # noqa: F401
from vdiff.unet_audio import AudioFeatureTransformer, UNetAudio, Wav2Vec2Encoder  # noqa: F401
