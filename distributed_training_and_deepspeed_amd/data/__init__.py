from .sampler import DeviceBatchLoader, DistributedSampler  # noqa: F401
from .synthetic import IGNORE_INDEX, NativeSyntheticLM, SyntheticLMDataset, load_synthetic, mlm_mask_tokens  # noqa: F401
from .text import TokenizedLMDataset, load_wikitext, read_text_lines  # noqa: F401
