"""Model families: the case5/case6 attention blocks and an attention+FF transformer layer."""
from .attention import MultiHeadAttention, attention_block_flops  # noqa: F401
from .transformer import TransformerLayer, transformer_layer_flops  # noqa: F401
from .mlp import DenseStack, dense_stack_flops, feed_forward_flops  # noqa: F401
