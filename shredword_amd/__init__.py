"""shredword_amd -- MI355X-native batched BPE encode behind shredword's tokenizer surface.

    from shredword_amd import Tokenizer
    tok = Tokenizer(device=0)
    tok.load("model.model")          # "shredword v1" file (shredword/base.py:135-149)
    ids = tok.encode("hello world")  # pre-split on host (C++), merge loop on the GPU (HIP)
"""
from .base import (BaseTokenizer, CL100K_PATTERN, GPT2_PATTERN, apply_regex, build_vocab, get_stats, merge,
                   render_token, replace_control_characters)
from .tokenizer import Tokenizer
from .trainer import BPETrainer

__version__ = "0.1.0"
__all__ = ["BaseTokenizer", "BPETrainer", "Tokenizer", "apply_regex", "build_vocab", "get_stats", "merge", "render_token",
           "replace_control_characters", "CL100K_PATTERN", "GPT2_PATTERN"]
