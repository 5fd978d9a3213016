"""The ViT-L/16 pre-training config's training keys (configs/train/vitl16/pretrain-256px-16f.yaml,
lines 1-98 of the reference), restated as a dict for the launcher tests: /root/reference does not
exist on the GPU box. `micro()` shrinks batch / crop / frames / schedule so a test finishes in
seconds; every other key keeps the config's value."""

import copy

MASK = dict(aspect_ratio=[0.75, 1.5], full_complement=False, max_keep=None, max_temporal_keep=1.0,
            temporal_scale=[1.0, 1.0])

VITL_PRETRAIN_256_16F = {
    "app": "vjepa",
    "folder": "/your_folder/pretrain/16.8.vitl.256px.16f",
    "data": {"dataset_type": "VideoDataset", "batch_size": 24, "crop_size": 256, "patch_size": 16,
             "dataset_fpcs": [16, 16, 16], "tubelet_size": 2, "fps": 4, "num_workers": 8,
             "persistent_workers": True, "pin_mem": True},
    "data_aug": {"auto_augment": False, "motion_shift": False, "random_resize_aspect_ratio": [0.75, 1.35],
                 "random_resize_scale": [0.3, 1.0], "reprob": 0.0},
    "loss": {"loss_exp": 1.0},
    "mask": [dict(MASK, num_blocks=8, spatial_scale=[0.15, 0.15]), dict(MASK, num_blocks=2, spatial_scale=[0.7, 0.7])],
    "meta": {"dtype": "bfloat16", "eval_freq": 100, "load_checkpoint": True, "read_checkpoint": None,
             "save_every_freq": 50, "seed": 239, "use_sdpa": True},
    "model": {"model_name": "vit_large", "pred_depth": 12, "pred_embed_dim": 384, "pred_num_heads": 12,
              "uniform_power": True, "use_activation_checkpointing": True, "use_mask_tokens": True,
              "use_rope": True, "zero_init_mask_tokens": True},
    "optimization": {"ema": [0.99925, 0.99925], "epochs": 10, "final_lr": 0.000525, "final_weight_decay": 0.04,
                     "ipe": 300, "ipe_scale": 1.25, "lr": 0.000525, "start_lr": 0.0001, "warmup": 40,
                     "weight_decay": 0.04},
}


def micro(folder, batch=2, crop=64, frames=8, ipe=2, epochs=1):
    cfg = copy.deepcopy(VITL_PRETRAIN_256_16F)
    cfg["folder"] = str(folder)
    cfg["data"].update(batch_size=batch, crop_size=crop, dataset_fpcs=[frames] * 3, num_workers=0)
    cfg["optimization"].update(ipe=ipe, epochs=epochs, warmup=0)
    cfg["meta"]["save_every_freq"] = -1
    return cfg
