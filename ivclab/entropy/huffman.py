"""ivclab.entropy.huffman (reference ivclab/entropy/huffman.py:5-53): host Huffman coder
in libivc (constriction is not needed)."""
from ivclab_amd.entropy.huffman import HuffmanCoder

__all__ = ["HuffmanCoder"]
