class LabelMultisetWrapper:
    def __init__(self, *args, **kwargs):
        raise NotImplementedError
