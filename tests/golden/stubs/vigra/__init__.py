from . import analysis, filters  # noqa
