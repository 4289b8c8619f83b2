"""Checkpoint format of train_utils/checkpoints.py:4-31 (unchanged keys)."""
import torch


def save_ckp(epoch, model, optimizer, lr_scheduler, train_loss, val_loss, cider_score, path):
    torch.save({"epoch": epoch, "model_state_dict": model.state_dict(),
                "optimizer_state_dict": optimizer.state_dict(),
                "lr_scheduler_state_dict": lr_scheduler.state_dict(), "train_loss": train_loss,
                "val_loss": val_loss, "cider_score": cider_score}, path)


def load_ckp(model, optimizer, lr_scheduler, path):
    checkpoint = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(checkpoint["model_state_dict"])
    optimizer.load_state_dict(checkpoint["optimizer_state_dict"])
    lr_scheduler.load_state_dict(checkpoint["lr_scheduler_state_dict"])
    return (checkpoint["epoch"], model, optimizer, lr_scheduler, checkpoint["train_loss"],
            checkpoint["val_loss"], checkpoint["cider_score"])
