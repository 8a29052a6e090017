"""One Loader output: where it comes from and which operations build it.

Resolution rules (the reference's PipelineSpec, ffcv/pipeline/pipeline_spec.py:8-50):

* ``source`` is a field name (decode that field) or an Operation of another
  pipeline (branch off its output; then no decoder of its own is allowed);
* a pipeline given as a plain list whose first element is an instance of
  the field's decoder class uses that element as the decoder; a list that
  starts with anything else gets the field's default decoder inserted;
* a field left out of ``pipelines`` gets the default decoder followed by
  ``ToTensor``;
* ``torch.nn.Module`` entries are wrapped in ``ModuleWrapper``.
"""
from typing import List, Union

import torch as ch

from .operation import Operation


class PipelineSpec:

    def __init__(self, source: Union[str, Operation], decoder: Operation = None,
                 transforms: List[Operation] = None):
        self.source = source
        self.decoder = decoder
        self.transforms = list(transforms or [])
        self.default_pipeline = decoder is None and not self.transforms and isinstance(source, str)

    def __repr__(self):
        return repr((self.source, self.decoder, self.transforms))

    __str__ = __repr__

    def accept_decoder(self, Decoder, output_name):
        from ..transforms.ops import ToTensor
        from ..transforms.module import ModuleWrapper
        if self.decoder is not None and not isinstance(self.source, str):
            raise ValueError("Source can't be a node and also have a decoder")
        if Decoder is not None:
            leading = self.transforms[0] if self.transforms else None
            if isinstance(leading, Decoder):
                self.decoder = self.transforms.pop(0)
            elif self.decoder is None:
                try:
                    self.decoder = Decoder()
                except Exception:
                    raise ValueError(f"Impossible to use default decoder for {output_name},"
                                     "make sure you specify one in your pipeline.")
        if self.default_pipeline:
            self.transforms.append(ToTensor())
        self.transforms = [ModuleWrapper(t) if isinstance(t, ch.nn.Module) else t for t in self.transforms]
