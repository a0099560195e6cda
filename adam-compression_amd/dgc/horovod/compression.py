"""Gradient compression interface of the patched Horovod front end
(dgc/horovod/compression.py:22-76): ``compress(tensor, name)`` / ``decompress(tensor, ctx)``."""
import torch

__all__ = ["Compressor", "NoneCompressor", "FP16Compressor", "Compression"]


class Compressor:
    """Interface for compressing and decompressing a given tensor."""

    @staticmethod
    def compress(tensor, name=None):
        """Returns the compressed tensor and the context needed to decompress it."""

    @staticmethod
    def decompress(tensor, ctx):
        """Inverse of ``compress``."""


class NoneCompressor(Compressor):
    """Identity (the default)."""

    @staticmethod
    def compress(tensor, name=None):
        return tensor, None

    @staticmethod
    def decompress(tensor, ctx):
        return tensor


class FP16Compressor(Compressor):
    """Floating-point tensors travel as fp16 and come back in their own dtype."""

    @staticmethod
    def compress(tensor, name=None):
        if tensor.dtype.is_floating_point:
            return tensor.type(torch.float16), tensor.dtype
        return tensor, tensor.dtype

    @staticmethod
    def decompress(tensor, ctx):
        return tensor.type(ctx) if ctx.is_floating_point else tensor


class Compression:
    """Available compressors."""
    none = NoneCompressor
    fp16 = FP16Compressor
