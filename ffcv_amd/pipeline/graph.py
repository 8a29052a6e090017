"""Per-field operator graph lowered to a HIP-stream schedule.

Replaces ffcv/pipeline/graph.py:232-487.  The reference builds a DAG of
decoder/transform nodes, groups them into alternating numba-JIT / Python
stages and generates stage functions with ``ast``.  Here:

1. ``Graph.__init__`` resolves decoders and builds the same node DAG
   (DecoderNode, TransformNode, RefNode semantics: graph.py:234-292).
2. ``lower()`` fuses the hot path: a RandomResizedCrop / CenterCrop decoder
   followed (through ToTensor / ToDevice / ToTorchImage) by Cutout,
   RandomHorizontalFlip and NormalizeImage(float16) becomes ONE device launch
   (crop draws + decode + resize + epilogue); the absorbed operations keep
   their state declarations but run as identities.
3. ``collect_requirements`` walks states exactly like graph.py:295-354.  A
   non-device-aware (user) operation that would receive device data gets an
   implicit device->host transfer in front of it, so reference-style numpy
   operations keep working; a pipeline that never asks for ToDevice ends
   with a transfer back to host, matching the reference's CPU output.
4. ``run`` executes the nodes in order on the slot's current HIP stream;
   device work is asynchronous, host operations run as plain Python.
"""
from collections import defaultdict
from dataclasses import replace
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch as ch

from .allocation_query import AllocationQuery, allocate_query
from .operation import Operation
from .pipeline_spec import PipelineSpec
from .state import State

INITIAL_STATE = State(jit_mode=True, device=ch.device('cpu'), dtype=np.dtype('u1'), shape=None)


class _ToHost(Operation):
    """Implicit device -> pinned host transfer (graph-inserted)."""
    device_aware = True
    per_sample = True

    def __init__(self, as_tensor=False):
        super().__init__()
        self.as_tensor = as_tensor

    def declare_state_and_memory(self, previous_state):
        dt = previous_state.dtype
        if self.as_tensor:
            return (replace(previous_state, jit_mode=False, device=ch.device('cpu')),
                    AllocationQuery(previous_state.shape, dt, ch.device('cpu')))
        np_dt = ch.empty((), dtype=dt).numpy().dtype if isinstance(dt, ch.dtype) else dt
        return (replace(previous_state, jit_mode=True, device=ch.device('cpu'), dtype=np_dt),
                AllocationQuery(previous_state.shape, np_dt))

    def generate_code(self):
        as_tensor = self.as_tensor

        def to_host(inp, dst):
            from . import runtime
            B = inp.shape[0]
            ctx = runtime.current()
            if isinstance(dst, np.ndarray):
                host = ch.from_numpy(dst[:B])
            else:
                host = dst[:B]
            host = host.view(inp.dtype) if host.dtype != inp.dtype else host
            if inp.dim() == host.dim() and tuple(inp.shape) != tuple(host.shape):
                host = host.reshape(inp.shape)
            host.copy_(inp, non_blocking=True)
            if ctx is not None and ctx.stream is not None:
                ctx.stream.synchronize()
            else:
                ch.cuda.synchronize()
            return host if as_tensor else dst[:B]
        return to_host


class Node:
    last_node_id = 0

    def __init__(self, operation, parent=None, field_name=None, f_ix=None):
        self.id = Node.last_node_id
        Node.last_node_id += 1
        self.operation = operation
        self.parent = parent
        self.field_name = field_name
        self.f_ix = f_ix
        self.code = None
        self.with_indices = False

    @property
    def is_decoder(self):
        return self.parent is None


class Graph:

    def __init__(self, pipeline_specs: Dict[str, PipelineSpec], handlers, fieldname_to_fix, metadata,
                 memory_read, device=None):
        self.memory_read = memory_read
        self.handlers = handlers
        self.fieldname_to_fix = fieldname_to_fix
        self.metadata = metadata
        self.pipeline_specs = pipeline_specs
        self.device = ch.device(device) if device is not None else ch.device('cpu')
        self.nodes: List[Node] = []
        self.leaf_nodes: Dict[str, Node] = {}
        self.operation_to_node = defaultdict(list)
        self._chains: Dict[str, List[Operation]] = {}

        for output_name, spec in pipeline_specs.items():
            if spec.source in self.handlers:
                field = self.handlers[spec.source]
                Decoder = field.get_decoder_class()
                spec.accept_decoder(Decoder, output_name)

        for output_name, spec in pipeline_specs.items():
            if spec.source is None:
                raise ValueError(f"Field {output_name} has no source")
            source = spec.source
            if isinstance(source, str):
                assert spec.decoder is not None
                node = Node(spec.decoder, None, source, fieldname_to_fix[source])
                self.operation_to_node[spec.decoder].append(node)
            else:
                entries = self.operation_to_node[source]
                if not entries:
                    raise ValueError(f"{source} not found in other pipelines")
                if len(entries) > 1:
                    raise ValueError(f"Reference to {source} ambiguous")
                node = entries[0]
            chain = [node.operation] if node.parent is None and isinstance(source, str) else []
            if isinstance(source, str):
                self.nodes.append(node)
            for operation in spec.transforms:
                node = Node(operation, node, node.field_name, node.f_ix)
                self.operation_to_node[operation].append(node)
                self.nodes.append(node)
                chain.append(operation)
            self.leaf_nodes[output_name] = node
            self._chains[output_name] = chain
        self.lower()
        self._finalized = False

    # ------------------------------------------------------------ fusion --
    def lower(self):
        from ..fields.rgb_image import ResizedCropRGBImageDecoder
        from ..transforms import (Cutout, RandomHorizontalFlip, NormalizeImage, ToTensor, ToDevice,
                                  ToTorchImage)
        if self.device.type != 'cuda':
            return
        for name, chain in self._chains.items():
            if not chain or not isinstance(chain[0], ResizedCropRGBImageDecoder):
                continue
            dec = chain[0]
            cutout = flip = norm = None
            cut_before_flip = False
            layout_changed = False
            for op in chain[1:]:
                if len(self.operation_to_node[op]) != 1:
                    break
                if isinstance(op, ToTensor):
                    continue
                if isinstance(op, ToTorchImage):
                    layout_changed = True
                    continue
                if isinstance(op, ToDevice):
                    t = ch.device(op.device)
                    if t.type == 'cuda' and (t.index is None or t.index == (self.device.index or 0)):
                        continue
                    break
                if isinstance(op, Cutout) and cutout is None and norm is None and not layout_changed:
                    cutout = op
                    cut_before_flip = flip is None
                    op._absorbed = True
                    continue
                if isinstance(op, RandomHorizontalFlip) and flip is None and norm is None \
                        and not layout_changed:
                    flip = op
                    op._absorbed = True
                    continue
                if isinstance(op, NormalizeImage) and norm is None and \
                        np.dtype(op.original_dtype) == np.float16 and \
                        np.asarray(op.lookup_table).shape == (256, 3):
                    norm = op
                    op._absorbed = True
                break
            dec.fuse(cutout=cutout, flip=flip, cutout_before_flip=cut_before_flip, normalize=norm)

    # ------------------------------------------------------ requirements --
    def _prepare(self, node: Node, op: Operation):
        field_name = node.field_name
        fix = self.fieldname_to_fix[field_name]
        op.accept_field(self.handlers[field_name])
        op.accept_globals(self.metadata[f'f{fix}'], self.memory_read)
        op._pipeline_device = self.device
        op._field_index = fix

    def collect_requirements(self):
        """Declare states node by node; insert host transfers where needed."""
        from ..transforms.ops import ToDevice
        states: Dict[int, State] = {}
        self.allocations: Dict[int, object] = {}
        self.exec_nodes: List[Node] = []
        node_out: Dict[int, Node] = {}
        has_todevice = {name: any(isinstance(o, ToDevice) for o in chain)
                        for name, chain in self._chains.items()}
        self.exec_parent: Dict[int, Optional[int]] = {}
        for node in self.nodes:
            op = node.operation
            self._prepare(node, op)
            if node.parent is None:
                state = INITIAL_STATE
                parent_id = None
            else:
                parent_id = node_out[node.parent.id].id
                state = states[parent_id]
                if state.device.type == 'cuda' and not getattr(op, 'device_aware', False):
                    tx = Node(_ToHost(), None, node.field_name, node.f_ix)
                    self._prepare(tx, tx.operation)
                    st, alloc = tx.operation.declare_state_and_memory(state)
                    states[tx.id] = st
                    self.allocations[tx.id] = alloc
                    self.exec_nodes.append(tx)
                    self.exec_parent[tx.id] = parent_id
                    parent_id = tx.id
                    state = st
            next_state, alloc = op.declare_state_and_memory(state)
            states[node.id] = next_state
            self.allocations[node.id] = alloc
            self.exec_nodes.append(node)
            self.exec_parent[node.id] = parent_id
            node_out[node.id] = node
        self.outputs = {}
        for name, leaf in self.leaf_nodes.items():
            out = node_out[leaf.id]
            st = states[out.id]
            if st.device.type == 'cuda' and not has_todevice.get(name, True):
                tx = Node(_ToHost(as_tensor=True), None, out.field_name, out.f_ix)
                self._prepare(tx, tx.operation)
                st2, alloc = tx.operation.declare_state_and_memory(st)
                states[tx.id] = st2
                self.allocations[tx.id] = alloc
                self.exec_nodes.append(tx)
                self.exec_parent[tx.id] = out.id
                out = tx
            self.outputs[name] = out
        self.states = states
        for n in self.exec_nodes:
            n.code = n.operation.generate_code()
            n.with_indices = bool(getattr(n.code, 'with_indices', False))
        self._finalized = True
        return self.allocations, {n.id: n.code for n in self.exec_nodes}

    def codegen_all(self, code=None):
        if not self._finalized:
            self.collect_requirements()
        return self.exec_nodes, [self.outputs[k].id for k in self.leaf_nodes]

    def groupable(self):
        """True when every operation treats samples independently, so that
        consecutive batches may run through the graph as one launch."""
        if not self._finalized:
            self.collect_requirements()
        return all(getattr(n.operation, 'per_sample', False) for n in self.exec_nodes)

    def allocation_signature(self):
        """The allocations in execution order, independent of node ids."""
        if not self._finalized:
            self.collect_requirements()

        def desc(q):
            if isinstance(q, AllocationQuery):
                return (tuple(int(x) for x in q.shape), str(q.dtype), str(q.device))
            if isinstance(q, Sequence):
                return tuple(desc(x) for x in q)
            return None
        return tuple((type(n.operation).__name__, desc(self.allocations[n.id])) for n in self.exec_nodes)

    def rebind_memory(self, memory):
        """Buffers allocated for an earlier collect_requirements() with the
        same allocation_signature(), re-keyed to the current node ids."""
        order = memory['__order__']
        new = {n.id: memory[old] for n, old in zip(self.exec_nodes, order)}
        new['__order__'] = [n.id for n in self.exec_nodes]
        return new

    def allocate_memory(self, batch_size, batches_ahead):
        if not self._finalized:
            self.collect_requirements()
        memory = {'__order__': [n.id for n in self.exec_nodes]}
        for node_id, q in self.allocations.items():
            if isinstance(q, AllocationQuery):
                memory[node_id] = allocate_query(q, batch_size, batches_ahead)
            elif isinstance(q, Sequence):
                memory[node_id] = tuple(allocate_query(x, batch_size, batches_ahead) for x in q)
            else:
                memory[node_id] = None
        return memory

    # ----------------------------------------------------------- execute --
    def run(self, batch_indices, storage_state, memory, slot):
        results = {}
        count = len(batch_indices)
        # the slot buffer views of one (memory, slot, count) never change:
        # built once instead of re-sliced every batch (host time per batch
        # is what bounds the Loader at the kernels' rate)
        sel = getattr(self, '_sel_cache', None)
        if sel is None or sel[0] is not memory:
            sel = self._sel_cache = (memory, {})
        mems = sel[1].get((slot, count))
        if mems is None:
            mems = sel[1][(slot, count)] = {n.id: select_buffer(memory[n.id], slot, count)
                                            for n in self.exec_nodes}
        for node in self.exec_nodes:
            mem = mems[node.id]
            pid = self.exec_parent[node.id]
            if pid is None:
                fix = self.fieldname_to_fix[node.field_name]
                res = node.code(batch_indices, mem, self.metadata[f'f{fix}'], storage_state)
            else:
                inp = results[pid]
                if node.with_indices:
                    res = node.code(inp, mem, batch_indices)
                else:
                    res = node.code(inp, mem)
            results[node.id] = res
        return tuple(results[self.outputs[k].id] for k in self.leaf_nodes)


def select_buffer(buffer, batch_slot, count):
    """epoch_iterator.py:22-30: the slot's sub-buffer for this batch."""
    if buffer is None:
        return None
    if isinstance(buffer, tuple):
        return tuple(select_buffer(x, batch_slot, count) for x in buffer)
    return buffer[batch_slot][:count]
