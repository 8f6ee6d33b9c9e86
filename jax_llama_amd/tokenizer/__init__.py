from .llama2 import Tokenizer as LLaMA2Tokenizer
from .llama3 import ChatFormat, Dialog, Message
from .llama3 import Tokenizer as LLaMA3Tokenizer

__all__ = ["LLaMA2Tokenizer", "LLaMA3Tokenizer", "ChatFormat", "Dialog", "Message"]
