def gaussianSmoothing(*args, **kwargs):
    raise NotImplementedError("sigma_prefilter is out of scope")
