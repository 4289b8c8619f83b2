"""Config with the reference template's attribute names and defaults
(configuration_template.py:4-57) plus optional MI355X build knobs:

* ``dtype``: 'bf16' (default; bf16 operands, fp32 accumulation/master weights) or 'fp32'
  (exact-f32 MFMA, the parity mode used against the reference CPU path).
* ``grad_bucket_mb``: data-parallel gradient bucket size.
* ``deterministic``: fixed-order reductions everywhere (no split-K fp32 atomics), so two runs
  on the same inputs give bitwise-equal gradients and weights (``retr_set_deterministic``).
"""
from os.path import join


class Config(object):
    def __init__(self):
        self.prefix = "refcoco"
        self.lr_backbone = 1e-5
        self.lr = 1e-4
        self.epochs = 30
        self.lr_drop = 20
        self.start_epoch = 0
        self.weight_decay = 1e-4
        self.backbone = "ResNet101"
        self.position_embedding = "sine"
        self.dilation = True
        self.device = "cuda"
        self.seed = 42
        self.batch_size = 32
        self.num_workers = 8
        self.checkpoint = f"./{self.prefix}_checkpoint.pth"
        self.project_data_path = "./data"
        self.checkpoint_path = join(self.project_data_path, "models", self.prefix)
        self.clip_max_norm = 0.1
        self.early_stopping = True
        self.use_global_features = False
        self.use_location_features = False
        self.verbose = True
        self.transformer_type = "Concat"
        self.hidden_dim = 256
        self.pad_token_id = 0
        self.max_position_embeddings = 128
        self.layer_norm_eps = 1e-12
        self.dropout = 0.1
        self.vocab_size = 30522
        self.enc_layers = 6
        self.dec_layers = 6
        self.dim_feedforward = 2048
        self.nheads = 8
        self.pre_norm = True
        self.dir = "PATH_TO_COCO"
        self.ref_base = "PATH_TO_REF_BASE"
        self.ref_dir = join(self.ref_base, self.prefix)
        self.limit = -1
        # MI355X build knobs (absent from reference configs -> defaults below)
        self.dtype = "bf16"
        self.grad_bucket_mb = 64
        self.deterministic = False


def compute_dtype(config):
    import torch
    name = getattr(config, "dtype", "bf16")
    if name in ("bf16", "bfloat16", torch.bfloat16):
        return torch.bfloat16
    if name in ("fp32", "float32", torch.float32):
        return torch.float32
    raise ValueError(f"unsupported dtype {name!r} (bf16|fp32)")
