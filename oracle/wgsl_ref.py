"""The reference's operators with their WGSL executed -- TEST INFRASTRUCTURE ONLY.

The host side of each operator is restated from the reference's Rust (cited
per method); the compute side is NOT restated: the reference's own shader
files are read from the reference checkout and executed by
``oracle/wgsl_exec.py`` under explicit pins for what WGSL leaves to the
implementation.  This pins the C oracle (``dips_oracle.c``) and the numpy
restatement to the shader text (tests/test_wgsl_pin.py) and generates the
``wgsl_*`` golden fixtures (tests/golden/make_wgsl_golden.py) that the GPU
tests run through the HIP path.

The reference checkout is only read here, in this container (the path is
``$DIPS_REFERENCE_ROOT``, default /root/reference).  No shader text is
copied into the repository; the fixtures record the sha256 of each shader
file they were generated from.
"""
from __future__ import annotations

import hashlib
import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from oracle.wgsl_exec import PINS, Module, Pins, Texture

REF_ROOT = os.environ.get("DIPS_REFERENCE_ROOT", "/root/reference")
DIPS_SHADER = "dips/src/gpu/shaders/dips_shader.wgsl"
DIPS_PRE_SHADER = "dips/src/gpu/shaders/pre_compute_shader.wgsl"
ALT_SHADER = "dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl"

WORK_GROUP = 16  # dips/src/gpu/mod.rs:19-20, dips_alt/src/dips_compute/mod.rs (same constants)
TEMPORAL_BUFFER_SIZE = 4  # dips/src/gpu/bind_groups.rs:18
ALT_FRAME_COUNT = 2  # dips_alt/src/lib.rs:36


def available() -> bool:
    return all(os.path.isfile(os.path.join(REF_ROOT, p)) for p in (DIPS_SHADER, DIPS_PRE_SHADER, ALT_SHADER))


def shader_text(rel: str) -> str:
    with open(os.path.join(REF_ROOT, rel)) as f:
        return f.read()


def shader_sha256(rel: str) -> str:
    with open(os.path.join(REF_ROOT, rel), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


_MODULES: Dict[str, Module] = {}


def module(rel: str, text: Optional[str] = None) -> Module:
    key = rel if text is None else rel + "#" + hashlib.sha256(text.encode()).hexdigest()
    if key not in _MODULES:
        _MODULES[key] = Module(shader_text(rel) if text is None else text)
    return _MODULES[key]


def _groups(width: int, height: int):
    """compute_work_group_count (dips/src/gpu/mod.rs:23-31)."""
    return ((width + WORK_GROUP - 1) // WORK_GROUP, (height + WORK_GROUP - 1) // WORK_GROUP, 1)


class ComputeState:
    """dips ComputeState (dips/src/gpu/mod.rs:39-398) over the executed
    shaders.  Filter codes as the reference's `Into<f64>` (lib.rs:26-60):
    Sigmoid 0, InverseSigmoid 1, Unfiltered 255; chroma None 0, R 1, G 2,
    B 3."""

    def __init__(self, colorize: bool, spatial_window_size: int, sensitivity: float, filter_type: int,
                 chroma_filter: int, pins: Pins = PINS):
        # the pipeline constants (gpu/mod.rs:101-109), f64 values
        consts = {"0": 1.0 if colorize else 0.0, "1": float(spatial_window_size),
                  "2": float(np.float32(sensitivity)), "3": float(filter_type), "4": float(chroma_filter)}
        # both modules get the same map (gpu/mod.rs:124, 145)
        self.pre = module(DIPS_PRE_SHADER).pipeline("pre_compute_main", consts, pins)
        self.main = module(DIPS_SHADER).pipeline("compute_main", consts, pins)
        self.textures: List[np.ndarray] = []   # the VecDeque (mod.rs:53, 170-176)
        self.starting_texture: Optional[np.ndarray] = None
        self.slots: Optional[List[Texture]] = None  # MainComputeBindGroups (bind_groups.rs:244-272)
        self.index = 0          # UCircularIndex (bind_groups.rs:371, indexing.rs:13-28)
        self.uniform = 0        # starting_temporal_index_buffer (bind_groups.rs:317-321, 419-424)
        self.dims = None

    def add_texture(self, width: int, height: int, frame_data) -> None:
        """mod.rs:170-216."""
        frame = np.asarray(frame_data, dtype=np.uint8).reshape(height, width, 4).copy()
        self.textures.append(frame)
        if len(self.textures) > TEMPORAL_BUFFER_SIZE:
            self.textures.pop(0)
        if len(self.textures) != TEMPORAL_BUFFER_SIZE:
            return
        if self.starting_texture is None:  # PreComputeBindGroups::initialize Ok -> run_precompute_pipeline
            self.dims = (width, height)
            out = Texture(np.zeros((height, width, 4), np.uint8))
            self.pre.dispatch({"start_texture_array": [Texture(t.copy()) for t in self.textures],
                               "output_texture": out}, _groups(width, height))
            self.starting_texture = out.data.copy()   # read back, de-padded (mod.rs:218-303)
        if self.slots is None:  # MainComputeBindGroups::initialize Ok (starting index 0)
            self.slots = [Texture(t.copy()) for t in self.textures]
            self.start = Texture(self.starting_texture.copy())  # set_start_texture (bind_groups.rs:376-387)
            self.index = 0
            self.uniform = 0
        else:  # update_temporal_texture (bind_groups.rs:407-427)
            self.slots[self.index] = Texture(frame.copy())
            self.uniform = self.index
            self.index = (self.index + 1) % TEMPORAL_BUFFER_SIZE

    def dispatch(self) -> Optional[np.ndarray]:
        """mod.rs:306-397: one dispatch, the output texture read back."""
        if self.slots is None:
            return None
        width, height = self.dims
        out = Texture(np.zeros((height, width, 4), np.uint8))
        self.main.dispatch({"start_texture": self.start, "temporal_texture_array": self.slots,
                            "starting_index": self.uniform, "output_texture": out}, _groups(width, height))
        return out.data.copy()

    def start_texture(self) -> Optional[np.ndarray]:
        return None if self.starting_texture is None else self.starting_texture.copy()


def frame_callback(width: int, height: int, frame, compute: ComputeState) -> np.ndarray:
    """dips/src/lib.rs:233-246."""
    compute.add_texture(width, height, frame)
    out = compute.dispatch()
    return out if out is not None else np.asarray(frame, np.uint8).reshape(height, width, 4).copy()


def alt_shader_text(num_textures: int) -> str:
    """The module dips_alt builds (dynamic_texture_array.rs:25-117): one
    `texture_<i>` binding per texture, the per-texture median_array lines and
    the `load_from_texture_id` switch cases spliced in at the two markers, the
    bindings prepended."""
    bindings, arraying, loading = "", "", ""
    group = 0
    for index in range(num_textures):
        if index % 4 == 0 and index != 0:
            group += 1
        bindings += f"@group({group}) @binding({index % 4})\nvar texture_{index}: texture_storage_2d<rgba8unorm, read>;\n"
        arraying += f"    median_array[{index}] = spatial_median_filter(coords.xy, dimensions.xy, {index});\n"
        loading += f"        case {index}u: {{\n            return textureLoad(texture_{index}, coords.xy);\n        }}\n"
    text = shader_text(ALT_SHADER)
    text = text.replace("//r3p1Ac3", arraying)
    text = text.replace("//lFtIr3p1Ac3", loading)
    return bindings + text


class AltCompute:
    """dips_alt DiPsCompute (dips_alt/src/dips_compute/mod.rs:243-647) over
    the executed shader.  width = frame columns, height = rows (the
    reference's constructor takes (rows, cols) and swaps them back,
    mod.rs:283-286, lib.rs:596-603)."""

    def __init__(self, num_textures: int, width: int, height: int, colorize: bool = True, window: int = 1,
                 scalar: float = 5.0, filter_type: int = 0, chroma: int = 0, pins: Pins = PINS):
        self.n = int(num_textures)
        self.width, self.height = int(width), int(height)
        # get_properties_hash_map (mod.rs:189-207) + NUM_TEXTURES (mod.rs:453)
        consts = {"COLORIZE": 1.0 if colorize else 0.0, "WINDOW_SIZE": float(window),
                  "SIGMOID_HORIZONTAL_SCALAR": float(np.float32(scalar)), "FILTER_TYPE": float(filter_type),
                  "CHROMA_FILTER": float(chroma), "NUM_TEXTURES": float(self.n)}
        text = alt_shader_text(self.n)
        self.pipe = module(ALT_SHADER, text).pipeline("pre_compute_main", consts, pins)
        # zero-initialised textures (wgpu clears new textures)
        self.inputs = [Texture(np.zeros((self.height, self.width, 4), np.uint8)) for _ in range(self.n)]
        self.snapshot_texture = Texture(np.zeros((self.height, self.width, 4), np.uint8))
        self.index = 0

    def send_frame(self, frame, snapshot: bool = False) -> np.ndarray:
        """mod.rs:498-646 (the no-renderer branch)."""
        self.inputs[self.index] = Texture(np.asarray(frame, np.uint8).reshape(self.height, self.width, 4).copy())
        self.index = (self.index + 1) % self.n
        out = Texture(np.zeros((self.height, self.width, 4), np.uint8))
        b = {f"texture_{i}": t for i, t in enumerate(self.inputs)}
        b.update({"snapshot": 1 if snapshot else 0, "snapshot_texture": self.snapshot_texture,
                  "output_texture": out})
        self.pipe.dispatch(b, _groups(self.width, self.height))
        return out.data.copy()

    def run(self, frames: Sequence[np.ndarray], markers=()) -> np.ndarray:
        """run_dips_on_file's loop (dips_alt/src/lib.rs:567-683): the snapshot
        on the FRAME_COUNT-th frame after the start or a refresh marker."""
        index, overall, outs = 0, 0, []
        for f in frames:
            outs.append(self.send_frame(f, snapshot=(index == ALT_FRAME_COUNT)))
            if index <= ALT_FRAME_COUNT:
                index += 1
            overall += 1
            if overall in markers:
                index = 0
        return np.stack(outs) if outs else np.zeros((0, self.height, self.width, 4), np.uint8)


def get_intensity(rgba: np.ndarray, chroma: int, pins: Pins = PINS) -> np.ndarray:
    """dips_shader.wgsl's get_intensity executed over an [N, 4] uint8 batch
    of texels (loaded as rgba8unorm)."""
    from oracle.wgsl_exec import V
    consts = {"4": float(chroma)}
    pipe = module(DIPS_SHADER).pipeline("compute_main", consts, pins)
    px = np.asarray(rgba, np.uint8).reshape(-1, 4)
    v = V(("vec", 4, "f32"), px.astype(np.float32) / np.float32(255.0))
    return np.asarray(pipe.call("get_intensity", [v]).d, dtype=np.float32)
