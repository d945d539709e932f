"""Drop-in for the reference's utils.py:1-39 (checkpoint helpers), with the
key mapping between the reference's tcnn modules and models.networks.NGP:

  reference state_dict (Lightning 'state_dict', prefix 'model.')   NGP here
  xyz_encoder.params  = [W1 64x32 | W2 16x64 | hash table]          params[:3072] + params[10240:]
  rgb_net.params      = [W3 64x32 | W4 64x64 | W5 16x64]            params[3072:10240]
  center, xyz_min, xyz_max, half_size, density_bitfield,            same-named buffers
  density_grid, grid_coords (train.py:79-82)                        buffers when present

Checkpoints are read with torch.load(weights_only=True): tensors and plain
containers only (a Lightning checkpoint whose hyper-parameters are pickled
objects is refused by the safe loader -- slim it first with the reference,
or save state_dict only, as ModelCheckpoint(save_weights_only=True) does).
"""
import torch

TCNN_KEYS = ("xyz_encoder.params", "rgb_net.params")
# tcnn modules without trainable state still register an (empty) `params`
# Parameter -- the SH dir_encoder (models/networks.py:59-66) -- so every
# reference checkpoint holds 'model.dir_encoder.params' of shape [0]
EMPTY_TCNN_KEYS = ("dir_encoder.params",)


def _load(ckpt_path):
    return torch.load(ckpt_path, map_location="cpu", weights_only=True)


def extract_model_state_dict(ckpt_path, model_name='model', prefixes_to_ignore=[]):
    """utils.py:4-18: the `model_name.`-prefixed entries, prefix stripped."""
    checkpoint = _load(ckpt_path) if isinstance(ckpt_path, str) else ckpt_path
    if 'state_dict' in checkpoint:  # a pytorch-lightning checkpoint
        checkpoint = checkpoint['state_dict']
    out = {}
    for k, v in checkpoint.items():
        if not k.startswith(model_name):
            continue
        k = k[len(model_name) + 1:]
        if any(k.startswith(p) for p in prefixes_to_ignore):
            continue
        out[k] = v
    return out


def tcnn_state_dict(model):
    """NGP state in the reference's key layout (loadable by its load_ckpt)."""
    sd = {k: v for k, v in model.state_dict().items() if k != 'params'}
    xyz, rgb = model.tcnn_params()
    sd['xyz_encoder.params'] = xyz.clone()
    sd['rgb_net.params'] = rgb.clone()
    sd['dir_encoder.params'] = torch.zeros(0, dtype=rgb.dtype)
    for name in ('density_grid', 'grid_coords'):
        if hasattr(model, name) and name not in sd:
            sd[name] = getattr(model, name)
    return sd


@torch.no_grad()
def load_ckpt(model, ckpt_path, model_name='model', prefixes_to_ignore=[]):
    """utils.py:21-26: update the model's state with the checkpoint's entries.
    tcnn-layout params (reference checkpoints) are mapped into NGP.params;
    density_grid / grid_coords are (re)registered as buffers like
    train.py:79-82 does before loading."""
    if not ckpt_path:
        return
    ck = extract_model_state_dict(ckpt_path, model_name, prefixes_to_ignore)
    if all(k in ck for k in TCNN_KEYS):
        model.load_tcnn_params(ck.pop(TCNN_KEYS[0]), ck.pop(TCNN_KEYS[1]))
    for k in EMPTY_TCNN_KEYS:  # parameter-free tcnn encodings: nothing to load
        if k in ck:
            if ck[k].numel() != 0:
                raise RuntimeError(f"checkpoint entry {k} should be empty, has {ck[k].numel()} values")
            ck.pop(k)
    for name in ('density_grid', 'grid_coords'):
        if name in ck and name not in dict(model.named_buffers()):
            if hasattr(model, name):
                delattr(model, name)
            model.register_buffer(name, torch.empty_like(ck[name]).to(model.density_bitfield.device))
    model_dict = model.state_dict()
    unknown = [k for k in ck if k not in model_dict]
    if unknown:
        raise RuntimeError(f"unexpected checkpoint keys for {type(model).__name__}: {unknown}")
    model_dict.update(ck)
    model.load_state_dict(model_dict)


def slim_ckpt(ckpt_path, save_poses=False):
    """utils.py:29-39: the Lightning state_dict without training-only entries."""
    ckpt = _load(ckpt_path) if isinstance(ckpt_path, str) else ckpt_path
    keys_to_pop = ['directions', 'model.density_grid', 'model.grid_coords']
    if not save_poses:
        keys_to_pop += ['poses']
    keys_to_pop += [k for k in ckpt['state_dict'] if k.startswith('val_lpips')]
    for k in keys_to_pop:
        ckpt['state_dict'].pop(k, None)
    return ckpt['state_dict']
