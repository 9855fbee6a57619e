"""Offline text loader (util.load_wikitext parity) with a tokenizer built in-process."""
import torch

from distributed_training_and_deepspeed_amd.data import IGNORE_INDEX, load_wikitext, read_text_lines


def _tokenizer(words):
    from tokenizers import Tokenizer, models, pre_tokenizers, processors
    from transformers import PreTrainedTokenizerFast
    specials = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    vocab = {t: i for i, t in enumerate(specials + sorted(set(words)))}
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    tok.post_processor = processors.TemplateProcessing(single="[CLS] $A [SEP]",
                                                       special_tokens=[("[CLS]", 2), ("[SEP]", 3)])
    return PreTrainedTokenizerFast(tokenizer_object=tok, pad_token="[PAD]", unk_token="[UNK]", cls_token="[CLS]",
                                   sep_token="[SEP]", mask_token="[MASK]", model_max_length=32)


def test_load_wikitext_mlm_and_causal(tmp_path):
    lines = [" ".join(f"w{(i * 7 + j) % 50}" for j in range(3 + i % 20)) for i in range(400)] + [""] * 20
    f = tmp_path / "wiki.train.raw"
    f.write_text("\n".join(lines) + "\n")
    assert len(read_text_lines(str(tmp_path))) == len(lines)
    tok = _tokenizer([w for ln in lines for w in ln.split()])
    ds = load_wikitext(tok, max_length=32, path=str(f), mlm=True, seed=1)
    assert ds.input_ids.shape == (len(lines), 32) and len(ds) == len(lines)
    lab = ds.labels
    special = (lab == IGNORE_INDEX)
    frac = (~special).float().sum() / (ds.input_ids != 0).float().sum()
    assert 0.08 < frac.item() < 0.2                      # ~15% of non-pad tokens (specials excluded)
    masked = ~special
    assert ((ds.input_ids == tok.mask_token_id) & masked).float().sum() / masked.float().sum() > 0.6
    c = load_wikitext(tok, max_length=32, path=str(f), mlm=False)
    assert torch.all(lab[c.input_ids == 0] == IGNORE_INDEX)    # pads never labelled under MLM
    assert torch.equal(c.labels, c.input_ids) and (c.labels == 0).any()   # causal: pads included (quirk 8)
    sub = ds.select(range(10))
    assert sub.input_ids.shape == (10, 32)
