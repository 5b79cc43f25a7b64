from .write import WriteLocal  # noqa: F401
