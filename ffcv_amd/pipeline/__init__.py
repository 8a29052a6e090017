from .pipeline_spec import PipelineSpec
from .compiler import Compiler
from .operation import Operation
from .state import State
from .allocation_query import AllocationQuery

__all__ = ['PipelineSpec', 'Compiler', 'Operation', 'State', 'AllocationQuery']
