"""ffcv_amd: MI355X-native drop-in for ffcv's image decode-and-augment path."""
__version__ = "0.1.0"
