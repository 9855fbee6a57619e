from .estimate import (MI355X_HBM_BYTES, ActivationCounter, activation_counter_hook, get_model_memory,  # noqa: F401
                       get_optimizer_memory, max_hidden_for_capacity, optimizer_bytes_per_param,
                       project_training_memory, project_transformer_memory, register_hooks_recursive)
