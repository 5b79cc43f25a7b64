"""luigi, or a minimal stand-in with the same surface when luigi is not installed.

luigi is the reference's workflow engine (cluster_tools/cluster_tasks.py:15); it is not
installed in this image.  The stand-in covers what the thresholded-components DAG uses:
Task (requires/output/run/complete, parameters as class attributes with defaults),
Parameter types, Target/LocalTarget and build(tasks, local_scheduler=True), which runs
the DAG depth-first and skips tasks whose output already exists (the reference's
checkpoint/resume behaviour, cluster_tasks.py:257-258).
"""
import os

try:  # pragma: no cover - exercised only where luigi exists
    import luigi as _luigi  # noqa: F401
    from luigi import (Task, Parameter, FloatParameter, IntParameter, ListParameter,  # noqa: F401
                       TaskParameter, BoolParameter, DictParameter, Target, LocalTarget, build)
    HAVE_LUIGI = True
except ImportError:
    HAVE_LUIGI = False

    class Parameter:
        _counter = 0

        def __init__(self, default=None, **kwargs):
            self.default = default
            Parameter._counter += 1
            self._order = Parameter._counter

        def normalize(self, v):
            return v

    class FloatParameter(Parameter):
        def normalize(self, v):
            return None if v is None else float(v)

    class IntParameter(Parameter):
        def normalize(self, v):
            return None if v is None else int(v)

    class BoolParameter(Parameter):
        def normalize(self, v):
            return bool(v)

    class ListParameter(Parameter):
        def normalize(self, v):
            return None if v is None else tuple(v)

    class DictParameter(Parameter):
        pass

    class TaskParameter(Parameter):
        pass

    class Target:
        def exists(self):
            return False

    class LocalTarget(Target):
        def __init__(self, path):
            self.path = path

        def exists(self):
            return os.path.exists(self.path)

    class Task:
        def __init__(self, **kwargs):
            params = {}
            for klass in reversed(type(self).__mro__):
                for k, v in vars(klass).items():
                    if isinstance(v, Parameter):
                        params[k] = v
            for k, p in params.items():
                if k in kwargs:
                    setattr(self, k, p.normalize(kwargs.pop(k)))
                elif p.default is not None or k not in kwargs:
                    setattr(self, k, p.default)
            if kwargs:
                raise TypeError('%s got unexpected parameters %s' % (type(self).__name__, sorted(kwargs)))

        def requires(self):
            return []

        def output(self):
            return None

        def input(self):
            req = self.requires()
            if isinstance(req, (list, tuple)):
                return [r.output() for r in req]
            return req.output() if req is not None else None

        def complete(self):
            out = self.output()
            if out is None:
                return False
            outs = out if isinstance(out, (list, tuple)) else [out]
            return all(o.exists() for o in outs)

        def run(self):
            pass

    def _deps(task):
        req = task.requires()
        if req is None:
            return []
        return list(req) if isinstance(req, (list, tuple)) else [req]

    def _run(task, seen):
        if id(task) in seen:
            return
        seen.add(id(task))
        for d in _deps(task):
            _run(d, seen)
        if not task.complete():
            task.run()

    def build(tasks, local_scheduler=True, **kwargs):
        """Run the DAGs; returns True on success (exceptions propagate as failure=False)."""
        try:
            for t in tasks:
                _run(t, set())
        except Exception as e:  # luigi reports failure instead of raising
            import traceback
            traceback.print_exc()
            build.last_exception = e
            return False
        return True
