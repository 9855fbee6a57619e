"""Built-in model configurations (no hub access on the MI355X boxes).

The reference pulls configs/weights from the HF hub
(``data_parallel_training.py:30-31``, ``model_parallel_training.py:36``,
``zero_dp_training.py:24``).  There is no network here, so every architecture the
reference trains is described by a built-in preset with random initialisation.
Parameter counts are checked in ``tests/test_models_cpu.py`` against the values
derived in SURVEY.md section 6 (bert-base MLM 108,340,804; bloom-560m 559,214,592;
opt-125m 125,239,296; gpt2-medium 354,823,168).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class TransformerConfig:
    name: str
    family: str  # "bert" | "bloom" | "opt" | "gpt2" | "block"
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    ffn_size: int
    max_positions: int = 512
    type_vocab_size: int = 0          # BERT token-type embeddings
    position_offset: int = 0          # OPT learned positions are offset by 2
    activation: str = "gelu"          # "gelu" (erf) | "gelu_tanh" | "relu"
    pre_ln: bool = False              # False = post-LN (BERT)
    causal: bool = False
    alibi: bool = False               # BLOOM ALiBi position bias
    embedding_ln: bool = False        # LN right after the embeddings (BERT, BLOOM)
    final_ln: bool = False            # final LN before the LM head (pre-LN models)
    mlm_head: bool = False            # BERT transform (dense+act+LN) + decoder bias
    tie_word_embeddings: bool = True
    ln_eps: float = 1e-5
    hidden_dropout: float = 0.1
    attn_dropout: float = 0.1
    bias: bool = True
    pad_token_id: int = 0
    special_token_ids: tuple = field(default_factory=tuple)
    mask_token_id: int = -1

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    def with_(self, **kw) -> "TransformerConfig":
        return replace(self, **kw)

    def to_dict(self) -> dict:
        return asdict(self)


# bert-base-cased / bert-large-cased (HF BertConfig defaults; special ids PAD 0, UNK 100,
# CLS 101, SEP 102, MASK 103 of the cased vocab) -- SURVEY.md D15/D19.
_BERT_SPECIAL = (0, 100, 101, 102, 103)

BERT_BASE = TransformerConfig(
    name="bert-base-cased", family="bert", vocab_size=28996, hidden_size=768, num_layers=12,
    num_heads=12, ffn_size=3072, max_positions=512, type_vocab_size=2, activation="gelu",
    pre_ln=False, causal=False, embedding_ln=True, mlm_head=True, ln_eps=1e-12,
    hidden_dropout=0.1, attn_dropout=0.1, pad_token_id=0, special_token_ids=_BERT_SPECIAL,
    mask_token_id=103,
)
BERT_LARGE = BERT_BASE.with_(name="bert-large-cased", hidden_size=1024, num_layers=24,
                             num_heads=16, ffn_size=4096)
# Small config for CPU/gloo plumbing tests (BASELINE config 1).
BERT_TINY = BERT_BASE.with_(name="bert-tiny", vocab_size=1024, hidden_size=128, num_layers=2,
                            num_heads=2, ffn_size=512, max_positions=512)

BLOOM_560M = TransformerConfig(
    name="bigscience/bloom-560m", family="bloom", vocab_size=250880, hidden_size=1024,
    num_layers=24, num_heads=16, ffn_size=4096, max_positions=2048, activation="gelu_tanh",
    pre_ln=True, causal=True, alibi=True, embedding_ln=True, final_ln=True, ln_eps=1e-5,
    hidden_dropout=0.0, attn_dropout=0.0, pad_token_id=3, special_token_ids=(0, 1, 2, 3),
)
OPT_125M = TransformerConfig(
    name="facebook/opt-125m", family="opt", vocab_size=50272, hidden_size=768, num_layers=12,
    num_heads=12, ffn_size=3072, max_positions=2048, position_offset=2, activation="relu",
    pre_ln=True, causal=True, final_ln=True, ln_eps=1e-5, hidden_dropout=0.1, attn_dropout=0.0,
    pad_token_id=1, special_token_ids=(0, 1, 2),
)
GPT2_MEDIUM = TransformerConfig(
    name="gpt2-medium", family="gpt2", vocab_size=50257, hidden_size=1024, num_layers=24,
    num_heads=16, ffn_size=4096, max_positions=1024, activation="gelu_tanh", pre_ln=True,
    causal=True, final_ln=True, ln_eps=1e-5, hidden_dropout=0.1, attn_dropout=0.1,
    pad_token_id=50256, special_token_ids=(50256,),
)
# Estimator block of estimate_transformer_memory.py:59-69 (OPT-style, h=9216, a=72, ffn 4h).
W4_BLOCK = TransformerConfig(
    name="w4-block", family="block", vocab_size=0, hidden_size=9216, num_layers=1, num_heads=72,
    ffn_size=36864, max_positions=512, activation="relu", pre_ln=True, causal=False,
    ln_eps=1e-5, hidden_dropout=0.1, attn_dropout=0.1,
)
CAUSAL_TINY = GPT2_MEDIUM.with_(name="causal-tiny", vocab_size=1024, hidden_size=128,
                                num_layers=2, num_heads=2, ffn_size=512, max_positions=512)

PRESETS = {
    c.name: c
    for c in (BERT_BASE, BERT_LARGE, BERT_TINY, BLOOM_560M, OPT_125M, GPT2_MEDIUM, W4_BLOCK,
              CAUSAL_TINY)
}
ALIASES = {
    "base": "bert-base-cased", "large": "bert-large-cased", "tiny": "bert-tiny",
    "bert-base": "bert-base-cased", "bert-large": "bert-large-cased",
    "bloom-560m": "bigscience/bloom-560m", "opt-125m": "facebook/opt-125m",
    "openai-community/gpt2-medium": "gpt2-medium",
}


def get_config(name: str) -> TransformerConfig:
    key = ALIASES.get(name, name)
    if key not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS) + sorted(ALIASES)}")
    return PRESETS[key]
