"""Minimal stand-in for luigi (absent here) so the reference's task modules import.

Test infrastructure only: used by tests/golden/make_golden.py to load the
reference job functions; never shipped, never on the GPU box.
"""


class Parameter:
    def __init__(self, *args, default=None, **kwargs):
        self.default = default


FloatParameter = IntParameter = ListParameter = TaskParameter = BoolParameter = DictParameter = Parameter


class Target:
    def exists(self):
        return False


class LocalTarget(Target):
    def __init__(self, path):
        self.path = path


class Task:
    def __init__(self, *args, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)
