class ResizedVolume:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("resized masks are out of scope")
