"""retr_amd — MI355X-native (gfx950) hot path of RE⫶TR (simeonjunker/retr).

Drop-in modules mirroring the reference package layout:
  retr_amd.models.caption.build_model      (models/caption.py)
  retr_amd.engine                          (engine.py)
  retr_amd.eval_utils.decode               (eval_utils/decode.py)
  retr_amd.train_utils.checkpoints         (train_utils/checkpoints.py)
  retr_amd.configuration.Config            (configuration_template.py)
``install_as_reference_modules()`` registers them under the reference's top-level names
(``models``, ``engine``, ``eval_utils``, ``train_utils``) so ``main.py`` / ``eval_model.py`` run
unchanged.
"""
import importlib
import sys

__all__ = ["install_as_reference_modules"]


def install_as_reference_modules():
    for name in ("models", "models.caption", "models.utils", "models.backbone",
                 "models.position_encoding", "models.transformer_modules",
                 "models.ConcatTransformer", "engine", "eval_utils", "eval_utils.decode",
                 "train_utils", "train_utils.checkpoints"):
        sys.modules[name] = importlib.import_module(f"retr_amd.{name}")
