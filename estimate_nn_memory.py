#!/usr/bin/env python
"""Parameter + activation memory of a small MLP (parity with the reference estimate_nn_memory.py).

Model memory = sum numel*element_size of parameters; activation memory = bytes of every
submodule's forward output (Dropout: 1-byte mask) plus the input tensor, which the hooks do
not see (reference :47-69).  Same demo: 4 Linear layers 512-1024-1024-1024-512 on batch 4.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_training_and_deepspeed_amd.memory import (ActivationCounter, get_model_memory,  # noqa: E402
                                                           register_hooks_recursive)


def main():
    model = torch.nn.Sequential(
        torch.nn.Linear(512, 1024),
        torch.nn.Linear(1024, 1024),
        torch.nn.Linear(1024, 1024),
        torch.nn.Linear(1024, 512),
    )
    print("Model Memory: {:,} bytes".format(get_model_memory(model)))
    counter = ActivationCounter()
    register_hooks_recursive(model, counter)
    inputs = torch.randn(4, 512)
    model(inputs)
    counter.add_activations(inputs)  # the hooks only capture layer outputs
    print("Activation Memory: {:,} bytes".format(counter.activation_bytes))
    return get_model_memory(model), counter.activation_bytes


if __name__ == "__main__":
    main()
