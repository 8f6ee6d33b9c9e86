from .engine import DecodeEngine, GenerateOutput, GenerationConfig, generate

__all__ = ["DecodeEngine", "GenerateOutput", "GenerationConfig", "generate"]
