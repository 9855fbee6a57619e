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


def test_device_batch_loader_prefetch_order_and_contents():
    """The one-ahead prefetching loader yields every sampler batch, in order, with the rows the
    sampler named (incl. the short last batch) -- CPU path; the side-stream path is exercised
    by the GPU trainers."""
    import torch

    from distributed_training_and_deepspeed_amd.data import DeviceBatchLoader, DistributedSampler

    class DS:
        def __init__(self, n):
            self.input_ids = torch.arange(n * 4).view(n, 4)
            self.labels = -self.input_ids

        def __len__(self):
            return self.input_ids.shape[0]

    ds = DS(11)
    sampler = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True, seed=5)
    order = list(iter(sampler))
    loader = DeviceBatchLoader(ds, batch_size=4, sampler=sampler)
    got = list(loader)
    assert len(got) == len(loader) == 3
    for i, b in enumerate(got):
        ix = torch.as_tensor(order[4 * i:4 * i + 4])
        assert torch.equal(b["input_ids"], ds.input_ids[ix]) and torch.equal(b["labels"], ds.labels[ix])
    assert list(DeviceBatchLoader(DS(0), batch_size=4)) == []
