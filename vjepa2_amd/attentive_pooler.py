"""Frozen-encoder probes (src/models/attentive_pooler.py): AttentivePooler and AttentiveClassifier
with the reference's constructor signatures, init RNG order and state_dict() keys, on the HIP
kernels — the self-attention Blocks (modules.Block without RoPE), the cross-attention of the learned
queries (modules.CrossAttentionBlock / CrossAttention -> vj_xattn) and the classifier Linear (HIP GEMM).
Forward and backward (the probe is what the reference's evals train on top of the frozen encoder).
"""

import math

import torch
import torch.nn as nn

from . import functions as fn
from .modules import Block, CrossAttention, CrossAttentionBlock, trunc_normal_


class AttentivePooler(nn.Module):
    """attentive_pooler.py:16-100."""

    def __init__(self, num_queries=1, embed_dim=768, num_heads=12, mlp_ratio=4.0, depth=1, norm_layer=nn.LayerNorm,
                 init_std=0.02, qkv_bias=True, complete_block=True, use_activation_checkpointing=False):
        super().__init__()
        self.use_activation_checkpointing = use_activation_checkpointing
        self.query_tokens = nn.Parameter(torch.zeros(1, num_queries, embed_dim))
        self.complete_block = complete_block
        if complete_block:
            self.cross_attention_block = CrossAttentionBlock(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio,
                                                             qkv_bias=qkv_bias, norm_layer=norm_layer)
        else:
            self.cross_attention_block = CrossAttention(dim=embed_dim, num_heads=num_heads, qkv_bias=qkv_bias)
        self.blocks = None
        if depth > 1:
            self.blocks = nn.ModuleList([
                Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias, qk_scale=False,
                      norm_layer=norm_layer) for _ in range(depth - 1)])
        self.init_std = init_std
        trunc_normal_(self.query_tokens, std=self.init_std)
        self.apply(self._init_weights)
        self._rescale_blocks()

    def _rescale_blocks(self):
        """attentive_pooler.py:65-76 (the cross block's fc2 takes the last block's layer id)."""
        layer_id = 0
        if self.blocks is not None:
            for layer_id, layer in enumerate(self.blocks):
                layer.attn.proj.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))
                layer.mlp.fc2.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))
        if self.complete_block:
            self.cross_attention_block.mlp.fc2.weight.data.div_(math.sqrt(2.0 * (layer_id + 1)))

    def _init_weights(self, m):
        """attentive_pooler.py:78-89."""
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=self.init_std)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)
        elif isinstance(m, nn.Conv2d):
            trunc_normal_(m.weight, std=self.init_std)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        """attentive_pooler.py:91-100: x [B, N, D] encoder tokens -> [B, num_queries, D] (f32)."""
        if self.blocks is not None:
            for blk in self.blocks:
                x = blk(x)  # activation checkpointing is not needed at probe sizes (HBM 288 GB)
        q = self.query_tokens.repeat(len(x), 1, 1)
        return self.cross_attention_block(q, x)


class AttentiveClassifier(nn.Module):
    """attentive_pooler.py:103-137."""

    def __init__(self, embed_dim=768, num_heads=12, mlp_ratio=4.0, depth=1, norm_layer=nn.LayerNorm, init_std=0.02,
                 qkv_bias=True, num_classes=1000, complete_block=True, use_activation_checkpointing=False):
        super().__init__()
        self.pooler = AttentivePooler(num_queries=1, embed_dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio,
                                      depth=depth, norm_layer=norm_layer, init_std=init_std, qkv_bias=qkv_bias,
                                      complete_block=complete_block,
                                      use_activation_checkpointing=use_activation_checkpointing)
        self.linear = nn.Linear(embed_dim, num_classes, bias=True)

    def forward(self, x):
        x = self.pooler(x).squeeze(1)
        return fn.run_linear(x, self.linear, out_dtype=torch.float32)
