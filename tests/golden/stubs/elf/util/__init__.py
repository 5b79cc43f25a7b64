def set_numpy_threads(n):
    pass
