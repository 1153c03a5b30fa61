"""Mirror of realtime_style_transfer/dataloaders/hdrScreenshots.py — Unreal HDR G-buffer screenshots.

A screenshot is ``<stem>.png`` (the final frame, used as ground truth) plus one EXR per G-buffer
channel, ``<stem>_<ChannelName>.exr`` (hdrScreenshots.py:16-18). ``expected_channels`` is the
``ShapeConfig.channels`` list of ``(name, num_channels)``.

* ``load_unreal_hdr_screenshot``            hdrScreenshots.py:14-30 — host (h, w, C) float32 array
* ``load_unreal_hdr_screenshot_to_device``  the hot-path variant: the channel planes go to the device
  as they are and ``rst_gbuffer_preprocess`` assembles, resizes and crops them in one pass (the host
  never concatenates or resizes)
* ``get_unreal_hdr_screenshot_dataset[_from_filepaths]``  hdrScreenshots.py:33-71 — an iterable
  dataset (seeded shuffle, log-and-skip on errors, optional ``output_shape`` ground truth) that
  decodes the next screenshot on a background thread while the caller consumes the current one
  (the reference's ``tf.data`` generator + ``prefetch``)
"""
from __future__ import annotations

import logging
import queue
import random
import threading
from pathlib import Path

import numpy as np
import torch

from . import exr
from .common import preprocess_numpy_image, preprocess_planes

log = logging.getLogger(__name__)


def _channel_paths(base_png_filepath: Path, expected_channels):
    base_png_filepath = Path(base_png_filepath)
    return [(base_png_filepath.parent / f"{base_png_filepath.stem}_{name}.exr", n) for name, n in expected_channels]


def _planes(exr_data, num_channels):
    if num_channels == 3:
        return [exr_data.channel('R'), exr_data.channel('G'), exr_data.channel('B')]
    if num_channels == 1:
        return [exr_data.channel('R')]
    return [c for _, c in exr_data.channels().items()]


def load_unreal_hdr_screenshot(base_png_filepath: Path, expected_channels):
    """hdrScreenshots.py:14-30: ((h, w, C) float32, base path)."""
    channel_list = []
    for path, n in _channel_paths(base_png_filepath, expected_channels):
        data = exr.load(str(path))
        if n in (1, 3):
            channel_list.append(np.stack(_planes(data, n), axis=-1))
        else:   # as the reference: np.stack over the channel dict (axis 0)
            channel_list.append(np.stack(_planes(data, n)))
    all_channels = np.concatenate(channel_list, axis=-1)
    log.debug(all_channels.shape)
    return all_channels, base_png_filepath


def load_unreal_hdr_screenshot_to_device(base_png_filepath: Path, expected_channels, shape, device=None,
                                         out: torch.Tensor = None) -> torch.Tensor:
    """Decode the channel EXRs and preprocess them on the device: (shape[0], shape[1], C), identical to
    ``preprocess_numpy_image(load_unreal_hdr_screenshot(...)[0], shape)``."""
    device = device or torch.device('cuda')
    planes = []
    for path, n in _channel_paths(base_png_filepath, expected_channels):
        if n not in (1, 3):
            raise ValueError(f"channel group {path.name}: only 1- and 3-channel groups are supported "
                             f"(the reference's stack for other counts is not channels-last)")
        for p in _planes(exr.load(str(path)), n):
            planes.append(torch.from_numpy(np.ascontiguousarray(p, dtype=np.float32)).to(device, non_blocking=False))
    return preprocess_planes(planes, shape, out=out)


def _load_ground_truth(png_path: Path, output_shape) -> torch.Tensor:
    """common.py:62-67 + 84-89: PIL lanczos load, cover-resize + center crop, /255 (host, PIL)."""
    import PIL.Image
    import math
    shape = output_shape[-3:]
    img = PIL.Image.open(png_path)
    img = img.convert('L' if shape[2] == 1 else 'RGB' if shape[2] == 3 else 'RGBA')
    tw, th = shape[1], shape[0]
    aspect_ratio_image = img.size[0] / img.size[1]
    aspect_ratio_target = tw / th
    if aspect_ratio_image > aspect_ratio_target:
        new_size = (math.ceil(th * aspect_ratio_image), th)
    else:
        new_size = (tw, math.ceil(tw / aspect_ratio_image))
    img = img.resize(new_size)
    width, height = img.size
    img = img.crop(((width - tw) / 2, (height - th) / 2, (width + tw) / 2, (height + th) / 2))
    a = np.asarray(img, dtype=np.float32).reshape(output_shape) / 255.0
    return torch.from_numpy(a)


class HdrScreenshotDataset:
    """Iterable over preprocessed screenshots (device tensors), decoded one ahead on a thread."""

    def __init__(self, screenshot_png_paths, expected_channels, shape, device=None, **kwargs):
        self.paths = list(screenshot_png_paths)
        if "seed" in kwargs:
            random.Random(kwargs['seed']).shuffle(self.paths)
        self.expected_channels = list(expected_channels)
        self.shape = tuple(shape)
        self.output_shape = kwargs.get('output_shape')
        self.device = device
        self.num_samples = len(self.paths)

    def _decode(self, png):
        planes = []
        for path, n in _channel_paths(png, self.expected_channels):
            planes += [np.ascontiguousarray(p, dtype=np.float32) for p in _planes(exr.load(str(path)), n)]
        gt = _load_ground_truth(png, self.output_shape) if self.output_shape is not None else None
        return planes, gt

    def __iter__(self):
        q: "queue.Queue" = queue.Queue(maxsize=2)
        done = object()

        def worker():
            for png in self.paths:
                try:
                    q.put((png, self._decode(png), None))
                except Exception as e:   # noqa: BLE001  (the reference logs and skips, hdrScreenshots.py:58-59)
                    q.put((png, None, e))
            q.put(done)

        threading.Thread(target=worker, daemon=True).start()
        dev = self.device or torch.device('cuda')
        while True:
            item = q.get()
            if item is done:
                return
            png, payload, err = item
            if err is not None:
                log.warning(f"Skipping f{png} due to an error: {err}")
                continue
            planes, gt = payload
            x = preprocess_planes([torch.from_numpy(p).to(dev) for p in planes], self.shape)
            yield (x, gt.to(dev)) if gt is not None else x

    def __len__(self):
        return self.num_samples


def get_unreal_hdr_screenshot_dataset_from_filepaths(screenshot_png_paths, expected_channels, shape, **kwargs):
    """hdrScreenshots.py:37-71."""
    return HdrScreenshotDataset(screenshot_png_paths, expected_channels, shape, **kwargs)


def get_unreal_hdr_screenshot_dataset(content_image_dir, expected_channels, shape, **kwargs):
    """hdrScreenshots.py:33-34: every ``*.png`` in ``content_image_dir``."""
    screenshot_pngs = list(Path(content_image_dir).glob('*.png'))
    return get_unreal_hdr_screenshot_dataset_from_filepaths(screenshot_pngs, expected_channels, shape, **kwargs)


__all__ = ["load_unreal_hdr_screenshot", "load_unreal_hdr_screenshot_to_device", "HdrScreenshotDataset",
           "get_unreal_hdr_screenshot_dataset", "get_unreal_hdr_screenshot_dataset_from_filepaths",
           "preprocess_numpy_image"]
