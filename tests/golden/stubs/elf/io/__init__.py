import h5py


def open_file(path, mode='a'):
    return h5py.File(path, mode)
