"""A detector view sharded over ranks, behind the reference's ``Workflow``
protocol (SRC/workflows/workflow_factory.py:22-34).

Event-batch sharding (SURVEY 8(e) axis 1): every rank runs its own
``GpuDetectorViewWorkflow`` (its own engine, LUT, window and cumulative) on
its share of the event messages.  The ranks call ``accumulate`` / ``finalize``
/ ``clear`` in the same sequence (SPMD, one process per GPU); what must agree
across ranks is kept in agreement by the wrapper:

* **Context** (the geometry signal ``detector_transform``, ROI requests and any
  other non-event keys) is taken from the root's ``accumulate`` call and
  shared in one small collective per batch, so every rank applies a detector
  move -- new LUT, cumulative reset (SRC/preprocessors/accumulators.py:
  116-131, SRC/workflows/geometry_signal.py:27-51) -- before binning the same
  batch.  A rank's own context keys are ignored: with sharding the root is
  the one context consumer.  The same collective tells every rank whether
  any rank has events in the batch, so the noise-replica cycle (one replica
  per batch, projectors.py:105-113) stays aligned when a rank's shard is
  empty.
* **clear()** is collective: every rank drops its window and cumulative.
* **finalize()** merges exactly: ``merge='outputs'`` RCCL-reduces every rank's
  uint64 partial images and totals onto the root (``OutputReducer``,
  2*S + 5 words); ``merge='window'`` reduces the windows (``WindowReducer``)
  so the root finalizes every output a single GPU would, including ROI
  spectra and spectrum views, which read the full histogram.  The root
  returns the reference's output dict; other ranks return ``None``.
* **float32 views** (BIFROST) merge per push (``merge='push'``, the default
  for them): the reference rounds its float32 accumulators once per push
  (SRC/preprocessors/accumulators.py:129-135, config/instruments/bifrost/
  specs.py:295), so the ranks' exact counts of every push are reduced onto
  the root (``PushReducer``) before the root adds them as one push; only the
  root's accumulators hold data and its finalize is a single workflow's.

Integer sums are order-independent, so the root's outputs are bit-identical
to one workflow that binned every rank's events.  ``root`` is a global rank,
also when ``group`` is a subgroup.
"""

from __future__ import annotations

from typing import Any, Iterable, Mapping

from .distributed import OutputReducer, PushReducer, WindowReducer
from .preprocessors import Timestamp
from .workflows import GpuDetectorViewWorkflow


class ShardedDetectorViewWorkflow:
    """``Workflow`` over the ranks of ``group`` (see the module doc)."""

    def __init__(self, workflow: GpuDetectorViewWorkflow, device, *, merge: str | None = None,
                 root: int = 0, group=None) -> None:
        import torch.distributed as dist

        eng = workflow.engine
        f32 = eng.dtype == 'float32'
        if merge is None:
            merge = 'push' if f32 else 'outputs'
        if merge not in ('outputs', 'window', 'push'):
            raise ValueError(f"merge must be 'outputs', 'window' or 'push', got {merge!r}")
        if f32 != (merge == 'push'):
            raise ValueError("float32 views merge per push (merge='push'), integer views at "
                             "finalize ('outputs' or 'window')")
        if merge == 'outputs' and workflow.has_grouped_outputs:
            raise ValueError("ROI spectra and spectrum views read the full histogram: use merge='window'")
        self._wf = workflow
        self._group = group
        self._root = root  # a global rank
        self._rank = dist.get_rank()
        self._is_root = self._rank == root
        self._merge = merge
        cls = {'outputs': OutputReducer, 'window': WindowReducer, 'push': PushReducer}[merge]
        self._reducer = cls(eng, device, dst=root, group=group)
        self._had_data = False  # this rank accumulated events since its last finalize

    @property
    def workflow(self) -> GpuDetectorViewWorkflow:
        return self._wf

    @property
    def is_root(self) -> bool:
        return self._is_root

    def build(self, *, context_keys: Mapping[str, Any] | None = None,
              chain_patch_bindings: Iterable = ()) -> None:
        self._wf.build(context_keys=context_keys, chain_patch_bindings=chain_patch_bindings)

    def _exchange(self, context: dict[str, Any], has_events: bool) -> tuple[dict[str, Any], bool]:
        """One collective: the root's context and whether any rank has
        events in this batch (the replica cycle advances once per batch with
        events, projectors.py:105-113, on every rank alike)."""
        import torch.distributed as dist

        world = dist.get_world_size(self._group)
        box: list = [None] * world
        dist.all_gather_object(box, (context if self._is_root else None, bool(has_events)),
                               group=self._group)
        root_index = dist.get_group_rank(self._group, self._root) if self._group is not None \
            else self._root
        return box[root_index][0] or {}, any(h for _, h in box)

    def accumulate(self, data: dict[str, Any], *, start_time: Timestamp,
                   end_time: Timestamp) -> None:
        """Collective.  ``data[source]`` holds this rank's event shard (may be
        absent); context keys come from the root."""
        source = self._wf.source_name
        context, any_events = self._exchange({k: v for k, v in data.items() if k != source},
                                             source in data)
        local = dict(context)
        if source in data:
            local[source] = data[source]
            self._had_data = True
        if self._merge != 'push':
            self._wf._accumulate(local, start_time, end_time, batch_has_events=any_events)
            return
        pushed = []

        def push(replica: int) -> None:
            self._reducer.push(replica)
            pushed.append(replica)

        self._wf._accumulate(local, start_time, end_time, batch_has_events=any_events, bin_fn=push)
        if any_events and not pushed:  # this rank has no share of the push
            self._reducer.push(0, has_events=False)

    def finalize(self) -> dict[str, Any] | None:
        """Collective.  The merged outputs on the root, ``None`` elsewhere."""
        had, self._had_data = self._had_data, False
        if self._merge == 'push':
            # every push was merged onto the root as it came
            if self._is_root:
                return self._wf.finalize()
            self._wf._end_window()
            return None
        if self._merge == 'window':
            root = self._reducer.reduce(had_data=had)
            if not root:
                # the window's counts moved to the root; this rank's cumulative
                # is never published, so it is dropped with the window
                self._wf.clear()
                self._wf._end_window()
                return None
            return self._wf.finalize()
        merged = self._reducer.finalize(had_data=had)
        if merged is None:
            self._wf._end_window()
            return None
        if not self._reducer.had_data:
            self._wf._end_window()
            raise ValueError('No data has been added')
        cur, cum, totals = merged
        return self._wf._outputs(cur, cum, totals)

    def clear(self) -> None:
        """Collective: every rank drops its window and cumulative."""
        import torch.distributed as dist

        dist.barrier(group=self._group)
        self._wf.clear()
        self._had_data = False
