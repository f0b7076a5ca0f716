"""Configuration: the reference's Hydra YAML keys, read with PyYAML.

Mirrors sres/base/util/config.py (ConfigContext, cfg()) closely enough that
the hot path reads the same keys from the same files:

* model:  config/model/<name>.yaml  -> nfeatures, nlayers, nblocks, cbottleneck,
          kernel_size, bias, downscale_factors, res_scale, batch_norm, loss_fn
* task:   config/task/<name>.yaml   -> batch_size, lr, weight_decay, tile_size,
          input_variables, target_variables, downsample_mode, upsample_mode
* pipeline.gpu / FMOD_GPU           -> device index (sres/base/gpu.py:6-15)

Parameter resolution follows init_parms (sres/model/common/common.py:9-28):
common defaults <- model-specific defaults <- kwargs, each overridden by the
model config when the key is present there.
Hydra/OmegaConf are not required (not installed on this image); when the code
runs inside a reference checkout, get_model() uses the reference's own cfg().
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, Iterable, List, Optional

import yaml

_HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(os.path.dirname(_HERE), "config")

COMMON_PARMS = dict(nchannels_in=1, nchannels_out=1, nfeatures=64, kernel_size=3, nlayers=16,
                    downscale_factors=[2, 2], bias=True, batch_norm=False, res_scale=1.0, ups_mode="bicubic",
                    # srmi's own key (absent from the reference yaml): the engine's operand type,
                    # "bf16" (bf16 MFMA operands, fp32 accumulate) or "fp32" (exact fp32)
                    dtype="bf16")
MODEL_PARMS = {"rcan": dict(cbottleneck=2, nblocks=20), "edsr": {}}


class Section(dict):
    """dict with attribute access and .get, like an OmegaConf DictConfig."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(d):
        if isinstance(d, dict):
            return Section({k: Section.wrap(v) for k, v in d.items()})
        return d


def search_paths() -> List[str]:
    paths = [CONFIG_DIR]
    extra = os.environ.get("SRMI_CONFIG_PATH")
    if extra:
        paths = extra.split(os.pathsep) + paths
    return paths


def load_group(group: str, name: str) -> Section:
    for root in search_paths():
        p = os.path.join(root, group, f"{name}.yaml")
        if os.path.exists(p):
            with open(p) as f:
                return Section.wrap(yaml.safe_load(f) or {})
    raise FileNotFoundError(f"config {group}/{name}.yaml not found in {search_paths()}")


class _Cfg(Section):
    pass


_CURRENT: Optional[_Cfg] = None


def cfg() -> _Cfg:
    if _CURRENT is None:
        raise RuntimeError("no active srmi ConfigContext")
    return _CURRENT


def _resolve_root(sec: Section) -> Section:
    """The platform yaml's relative interpolations (``${.root}/results``,
    ``{root}/results``; config/platform/*.yaml) resolved against its own root."""
    root = sec.get("root")
    if root is None:
        return sec
    for k, v in list(sec.items()):
        if isinstance(v, str) and k != "root":
            sec[k] = v.replace("${.root}", str(root)).replace("{root}", str(root))
    return sec


class ConfigContext:
    """with ConfigContext('sres', dict(task='SST-tiles-48', model='rcan-10-20-64', dataset='swot'), **{'task.lr': 1e-4}):

    Identity keys as the reference's ConfigContext.activate sets them
    (sres/base/util/config.py:51, :82-84): ``task.name`` = the task config name,
    ``task.dataset`` = the dataset config name and ``task.training_version`` =
    ``'-'.join([name, model, dataset, task])`` -- the stem of the checkpoint files
    (checkpoints.py:62) -- plus ``.model/.task/.dataset/.cid`` attributes on the
    context (ResultsAccumulator reads cc.dataset / cc.task / cc.model,
    manager.py:185-191)."""

    def __init__(self, cname: str, configuration: Dict[str, str], **overrides):
        self.cname = cname
        self.name = cname
        self.configuration = dict(configuration)
        self.overrides = overrides
        self.model = self.configuration.get("model")
        self.task = self.configuration.get("task")
        self.dataset = self.configuration.get("dataset")
        self.pipeline = self.configuration.get("pipeline")
        self.platform = self.configuration.get("platform")
        # config.py:51 joins the four names; the reference raises there when one is
        # missing.  A partial context (no dataset, say) is allowed here for the
        # hot-path plumbing, but it gets NO id: task.training_version stays unset, so
        # naming a checkpoint from it raises (CheckpointStore.from_config) instead of
        # silently using a name no reference run would write.
        names = (cname, self.model, self.dataset, self.task)
        self.cid = "-".join(str(v) for v in names) if all(v is not None for v in names) else None
        # the round-1..2 stem '{cname}-{model}': a resume that finds no checkpoint
        # under the reference name but one under this stem warns (harness.py)
        self.legacy_version = f"{cname}-{self.model}" if self.model is not None else None
        self._prev = None

    def load(self) -> _Cfg:
        c = _Cfg()
        for group, name in self.configuration.items():
            try:
                c[group] = load_group(group, name)
            except FileNotFoundError:
                c[group] = Section()
        c.setdefault("pipeline", Section(gpu=0))
        c.setdefault("task", Section())
        c.setdefault("model", Section())
        if "platform" in c:
            _resolve_root(c["platform"])
        for k, v in self.overrides.items():
            sec, key = k.split(".", 1)
            c.setdefault(sec, Section())[key] = v
        if "FMOD_GPU" in os.environ:  # sres/base/util/config.py:79
            c["pipeline"]["gpu"] = int(os.environ["FMOD_GPU"])
        # activate(), config.py:82-84
        if self.task is not None:
            c["task"]["name"] = self.task
        if self.dataset is not None:
            c["task"]["dataset"] = self.dataset
        if self.cid is not None:
            c["task"]["training_version"] = self.cid
        if self.legacy_version is not None:
            c["task"]["legacy_training_version"] = self.legacy_version
        return c

    def __enter__(self):
        global _CURRENT
        self._prev = _CURRENT
        _CURRENT = self.load()
        return _CURRENT

    def __exit__(self, *exc):
        global _CURRENT
        _CURRENT = self._prev
        return False


def model_section_from_env() -> Optional[Any]:
    """The active model config: the reference's cfg().model when running inside a
    reference checkout (plugin use), else srmi's own context, else None."""
    try:
        from sres.base.util.config import cfg as ref_cfg  # type: ignore
        return ref_cfg().model
    except Exception:
        pass
    if _CURRENT is not None:
        return _CURRENT.get("model")
    return None


def init_parms(model: str, custom: Dict[str, Any], model_cfg: Optional[Any] = None) -> Dict[str, Any]:
    """init_parms of sres/model/common/common.py:22-28."""
    mc = model_cfg if model_cfg is not None else model_section_from_env()
    get = (lambda k, d: mc.get(k, d)) if mc is not None else (lambda k, d: d)
    parms = {k: get(k, v) for k, v in COMMON_PARMS.items()}
    parms["scale"] = int(math.prod(list(parms["downscale_factors"])))
    for pd in (MODEL_PARMS.get(model, {}), custom):
        for k, v in pd.items():
            parms[k] = get(k, v)
    return parms


def data_downsample_factor(task):
    """apply_network's pre-downsampling of the HR batch (dual_trainer.py:561-563):
    ``downsample(input, scale_factor=ds)`` -- F.interpolate(scale_factor=1/ds,
    mode=torch_interp_mode(True)), array.py:72-76 -- only when ds > 1.0; any value
    <= 1 is a no-op there and here (returns 1).  Any factor > 1: an integer is
    returned as int, anything else as float (srmi.engine.downsample runs both)."""
    ds = float(task.get("data_downsample", 1.0) or 1.0) if task is not None else 1.0
    if ds <= 1.0:
        return 1
    return int(ds) if ds.is_integer() else ds


# torch_interp_mode (sres/base/util/array.py:37-41): 'linear' -> 'bilinear', 'cubic'
# -> 'bicubic', any other name passed to F.interpolate unchanged
_INTERP_NAMES = {"linear": "bilinear", "cubic": "bicubic", "bilinear": "bilinear", "bicubic": "bicubic"}


def interp_mode(task, downsample: bool) -> str:
    """The F.interpolate mode of downsample (task.downsample_mode) or upsample
    (task.upsample_mode), as torch_interp_mode maps them (array.py:37-41).  Absent
    keys mean 'cubic' (every reference task yaml sets cubic).  The engine runs
    'bilinear' and 'bicubic'; any other mode (e.g. 'nearest', 'area') raises
    NotImplementedError instead of silently resampling differently."""
    key = "downsample_mode" if downsample else "upsample_mode"
    mode = task.get(key, "cubic") if task is not None else "cubic"
    mode = "cubic" if mode is None else str(mode)
    if mode not in _INTERP_NAMES:
        raise NotImplementedError(f"task.{key}={mode!r}: srmi implements 'linear' (bilinear) and 'cubic' (bicubic)")
    return _INTERP_NAMES[mode]


def check_fused_task(task, nchannels_in: int, nchannels_out: int) -> Optional[List[int]]:
    """What the fused trainer takes from apply_network (dual_trainer.py:557-571).

    * ``task.data_downsample`` (:561-563): ``data_downsample_factor`` (the trainer
      downsamples the HR batch by it first).
    * ``task.downsample_mode`` / ``task.upsample_mode`` (array.py:37-41): validated
      by ``interp_mode`` (bilinear / bicubic; anything else raises).
    * The target channels: when the batch has MORE channels than
      ``task.target_variables`` the reference index_selects them (:564-568) with
      ``np.in1d(channels, target_variables).nonzero()`` -- the input's own order.
      Returned as that index list (the trainer selects the same channels of the HR
      batch on the device); None when nothing is selected (equal counts, whatever
      the order, are a no-op in the reference).  Without variable names the counts
      alone decide: fewer output channels than inputs cannot be resolved, and raise.
    """
    data_downsample_factor(task)
    interp_mode(task, True)
    interp_mode(task, False)
    names_in = list(task["input_variables"]) if task is not None and "input_variables" in task else None
    names_out = list(task["target_variables"]) if task is not None and "target_variables" in task else None
    if names_in is None or names_out is None:
        if nchannels_in != nchannels_out:
            raise NotImplementedError(f"target channel subset ({nchannels_out} of {nchannels_in} input variables) "
                                      "needs task.input_variables and task.target_variables")
        return None
    if len(names_in) != nchannels_in:
        raise ValueError(f"model has {nchannels_in} input channels, task.input_variables {names_in}")
    if len(names_in) <= len(names_out):
        if nchannels_out != nchannels_in:
            raise ValueError(f"model has {nchannels_out} output channels for target_variables {names_out}")
        return None
    idx = [i for i, v in enumerate(names_in) if v in set(names_out)]
    if len(idx) != nchannels_out:
        raise ValueError(f"target_variables {names_out} select {len(idx)} of the input channels {names_in}; "
                         f"the model has {nchannels_out} output channels")
    return idx


def tile_sizes(task) -> tuple:
    ts = task.get("tile_size", {"x": 48, "y": 48}) if task is not None else {"x": 48, "y": 48}
    return int(ts["y"]), int(ts["x"])
