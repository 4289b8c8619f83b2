"""CPU-side checks: C-ABI library loads and exports every declared symbol, drop-in API
(state_dict keys, freeze policy, error behaviour), no CPU fallback, synthetic inputs."""
import os
import re

import pytest
import torch

from retr_amd import _lib
from retr_amd.configuration import Config
from retr_amd.models.caption import build_model
from retr_amd.models.utils import NestedTensor, generate_square_subsequent_mask
from retr_amd.synthetic import synthetic_captions, synthetic_images, synthetic_state_dict
from tests.helpers import make_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "retr_hip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"\b(retr_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header_symbols():
    lib = _lib.load()
    assert lib.retr_abi_version() == 1
    for sym in declared_symbols():
        assert hasattr(lib, sym), sym
    assert set(declared_symbols()) == set(_lib.exported_symbols())


def test_state_dict_matches_reference_layout():
    c = make_config(backbone="ResNet50", hidden=256, layers=(6, 6), vocab=30522, max_pos=128,
                    ffn=2048)
    m, crit = build_model(c)
    sd = m.state_dict()
    assert len(sd) == 462
    assert "transformer.positional_encoding.pe" in sd
    assert sd["transformer.positional_encoding.pe"].shape == (1024, 1, 256)
    assert "backbone.body.layer4.2.bn3.running_var" in sd
    trainable = sum(p.numel() for p in m.parameters() if p.requires_grad)
    assert trainable == 65019962
    frozen = [n for n, p in m.named_parameters() if not p.requires_grad]
    assert all(("layer2" not in n and "layer3" not in n and "layer4" not in n) for n in frozen)
    assert all(n.startswith("backbone.") for n in frozen)


def test_build_model_errors_like_reference():
    c = make_config()
    c.use_global_features, c.use_location_features = True, False
    with pytest.raises(NotImplementedError):
        build_model(c)
    c = make_config()
    c.position_embedding = "bogus"
    with pytest.raises(ValueError):
        build_model(c)
    c = make_config(backbone="ResNet18", dilation=True)
    with pytest.raises(NotImplementedError):
        build_model(c)


def test_no_cpu_fallback():
    c = make_config()
    m, crit = build_model(c)
    img, mask = synthetic_images(1, 64)
    caps, cm = synthetic_captions(1, 16, 1000)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(NestedTensor(img, mask), caps[:, :-1], cm[:, :-1])


def test_synthetic_inputs_deterministic():
    c = make_config()
    m, _ = build_model(c)
    a = synthetic_state_dict(m, seed=3)
    b = synthetic_state_dict(m, seed=3)
    assert all(torch.equal(a[k], b[k]) for k in a)
    caps, cm = synthetic_captions(4, 128, 30522, seed=5)
    assert caps.shape == (4, 129) and (caps[:, 0] == 101).all()
    assert torch.equal(cm, caps == 0)


def test_causal_mask_helper():
    m = generate_square_subsequent_mask(4)
    assert torch.equal(torch.isinf(m), torch.ones(4, 4, dtype=torch.bool).triu(1))
    assert (m[~torch.isinf(m)] == 0).all()


def test_config_defaults_match_template():
    c = Config()
    assert (c.hidden_dim, c.enc_layers, c.dec_layers, c.nheads, c.dim_feedforward) == \
        (256, 6, 6, 8, 2048)
    assert (c.max_position_embeddings, c.vocab_size, c.layer_norm_eps) == (128, 30522, 1e-12)


def test_install_as_reference_modules_routes_reference_imports():
    """main.py / eval_model.py import `models.caption`, `engine`, `eval_utils.decode`,
    `train_utils.checkpoints` (main.py:1-12, eval_model.py:1-20): after the install those
    names resolve to the MI355X modules."""
    import sys
    import retr_amd
    names = ("models", "models.caption", "models.utils", "models.backbone",
             "models.position_encoding", "models.transformer_modules",
             "models.ConcatTransformer", "engine", "eval_utils", "eval_utils.decode",
             "train_utils", "train_utils.checkpoints")
    saved = {n: sys.modules.get(n) for n in names}
    try:
        retr_amd.install_as_reference_modules()
        import models.caption as mc
        import engine as eng
        from eval_utils.decode import greedy_decoding
        from train_utils.checkpoints import save_ckp, load_ckp  # noqa: F401
        import retr_amd.models.caption
        import retr_amd.engine
        import retr_amd.eval_utils.decode as dec
        assert mc is retr_amd.models.caption and eng is retr_amd.engine
        assert greedy_decoding is dec.greedy_decoding
        model, crit = mc.build_model(make_config())
        assert type(model).__name__ == "Caption"
    finally:
        for n, m in saved.items():
            if m is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = m


def test_prune_cap_ids_product_matches_oracle():
    from oracle import model as orc
    from retr_amd.eval_utils.decode import prune_cap_ids
    seqs = [[101, 5, 6, 102, 7, 0], [101, 0, 9, 9], [101, 102, 102], [], [3, 102]]
    for clean in (True, False):
        assert prune_cap_ids(seqs, clean, 0, 101, 102) == \
            orc.prune_cap_ids(seqs, clean, 0, 101, 102)


def test_tune_knob_table_matches_header_and_bad_env_is_skipped():
    """retr_amd._lib.TUNE_COUNT is the header's RETR_TUNE_COUNT, and a malformed or unknown
    RETR_TUNE_<n> environment preset is reported and skipped instead of breaking the import
    (ADVICE r5)."""
    import re
    import subprocess
    import sys
    from retr_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "retr_hip.h")).read()
    assert int(re.search(r"RETR_TUNE_COUNT = (\d+)", hdr).group(1)) == _lib.TUNE_COUNT
    code = ("import warnings; warnings.simplefilter('always'); "
            "from retr_amd import _lib; _lib.load(); print('loaded')")
    env = dict(os.environ, RETR_TUNE_7="abc", RETR_TUNE_99="1", RETR_TUNE_3="")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "loaded" in r.stdout
    assert "RETR_TUNE_7" in r.stderr and "RETR_TUNE_99" in r.stderr and "RETR_TUNE_3" in r.stderr


def test_kernel_family_classifier_covers_current_kernel_names():
    """bench.py / tools/pmc_*.py / tools/rocprof_families.py put every rocprof kernel name into a
    family with retr_amd.probe.family_of_symbol: the direct 3x3 conv's template (tile, row
    bytes, weight stages, direction) in both the mangled and the demangled spelling."""
    from retr_amd.probe import family_of_symbol
    mangled = ("_ZN12_GLOBAL__N_114conv3x3_kernelILi8ELi16ELi128ELi4ELi2ELi160ELi2ELb{}EN4retr6"
               "EpiFwdIDF16bDF16bEEEEvPKDF16bS5_T7_iiiiiii")
    assert family_of_symbol(mangled.format(0)) == "conv_fwd"
    assert family_of_symbol(mangled.format(1)) == "conv_dgrad"
    assert family_of_symbol("void (anonymous namespace)::conv3x3_kernel<8, 20, 128, 2, 4, 160, 3, "
                            "true, retr::EpiDgrad<bf16, bf16, bf16> >(...)") == "conv_dgrad"
    assert family_of_symbol("_ZN4retr12gemm2_kernelILi3ELi64ELi64E") == "conv_fwd"
    assert family_of_symbol("_ZN4retr17gemm_short_kernelILi0ELi64ELi64ELi4E") == "linear_fwd"
    assert family_of_symbol("retr::gemm_short_kernel<1, 32, 64, 4, x>(...)") == "linear_dgrad"
    assert family_of_symbol("conv_wgrad_group_kernel<1, 8, 128>") == "conv_wgrad"
    assert family_of_symbol("adamw_update_kernel<true>") is None
