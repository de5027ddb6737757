"""The reference's own end-to-end outputs, reproduced by the GPU build through
its drop-in host (iterative_cleaner_amd/cleaner.py):

* ``main()`` on the CLI fixture (iterative_cleaner.py:45-62, :148-157,
  :308-335): output naming, final weights after find_bad_parts, and stdout
  byte for byte (tests/golden/cli_case.npz, written by running the reference);
* ``main()`` with ``--memory -o`` on a 4-pol archive (tests/golden/cli_memory_case.npz)
  and with ``-o std`` (the NAME.FREQ.MJD.ar name, tests/golden/cli_std_name_case.npz);
* ``clean()`` with ``-z``: the zap PNG is pixel-identical to the reference's
  (iterative_cleaner.py:164-171; tests/golden/zap_plot_case.npz)."""
import hashlib
import os

import numpy as np
import pytest

from helpers import GOLDEN, bits_equal

pytestmark = pytest.mark.gpu


def test_cli_main_matches_reference(tmp_path, monkeypatch, capsys):
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    z = np.load(os.path.join(GOLDEN, "cli_case.npz"))
    data, weights, shift = synth.make_cube(10, 40, 128, 21, 0.2)
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"])
    wd = str(tmp_path)
    path = os.path.join(wd, "cli.ar")
    ica.Archive(data, weights, shift, filename=path).unload(path)
    monkeypatch.chdir(tmp_path)
    cleaner.main(cleaner.parse_arguments(["-l", "--bad_chan", "0.3", "--bad_subint", "0.3",
                                          "-c", "3", "-s", "3", path]))
    printed = capsys.readouterr().out.replace(wd, "<WD>")
    assert printed == str(z["stdout"])
    out_ar = ica.Archive_load(os.path.join(wd, "cli_cleaned.ar"))
    assert bits_equal(out_ar.get_weights(), z["weights"])


def test_cli_memory_output_matches_reference(tmp_path, monkeypatch, capsys):
    """main() with --memory and -o on a 4-pol archive (iterative_cleaner.py:66-70,
    :147-149): the named output keeps its 4 polarisations (neither pscrunched in
    memory nor reloaded) with the reference's weights, data bytes and stdout
    (tests/golden/cli_memory_case.npz)."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    z = np.load(os.path.join(GOLDEN, "cli_memory_case.npz"))
    data, weights, shift = synth.make_cube(6, 32, 64, 23, 0.2, npol=4)
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"])
    wd = str(tmp_path)
    path = os.path.join(wd, "mem.ar")
    ica.Archive(data, weights, shift, filename=path).unload(path)
    monkeypatch.chdir(tmp_path)
    cleaner.main(cleaner.parse_arguments(["-l", "--memory", "-o", "mem_out.ar", path]))
    printed = capsys.readouterr().out.replace(wd, "<WD>")
    assert printed == str(z["stdout"])
    out_ar = ica.Archive_load(os.path.join(wd, "mem_out.ar"))
    out = np.ascontiguousarray(out_ar.get_data())
    assert out.shape == tuple(z["data_shape"])
    assert bits_equal(out_ar.get_weights(), z["weights"])
    assert hashlib.sha256(out.tobytes()).hexdigest() == str(z["data_sha256"])


def test_cli_std_output_name_matches_reference(tmp_path, monkeypatch):
    """main() with -o std -q: the reference's NAME.FREQ.MJD.ar name
    (iterative_cleaner.py:52-56) and weights (tests/golden/cli_std_name_case.npz)."""
    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    z = np.load(os.path.join(GOLDEN, "cli_std_name_case.npz"))
    data, weights, shift = synth.make_cube(5, 16, 64, 24, 0.2)
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"])
    wd = str(tmp_path)
    path = os.path.join(wd, "std.ar")
    ica.Archive(data, weights, shift, filename=path).unload(path)
    monkeypatch.chdir(tmp_path)
    cleaner.main(cleaner.parse_arguments(["-l", "-q", "-o", "std", path]))
    names = sorted(f for f in os.listdir(wd) if f != "std.ar")
    assert names == [str(z["name"])]
    assert bits_equal(ica.Archive_load(os.path.join(wd, names[0])).get_weights(), z["weights"])


def test_zap_png_matches_reference(tmp_path, monkeypatch):
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    from iterative_cleaner_amd import archive as ica
    from iterative_cleaner_amd import cleaner, synth
    z = np.load(os.path.join(GOLDEN, "zap_plot_case.npz"))
    data, weights, shift = synth.make_cube(8, 24, 64, 61, 0.2)
    assert hashlib.sha256(data.tobytes()).hexdigest() == str(z["input_sha256"])
    monkeypatch.chdir(tmp_path)
    ica.Archive(data, weights, shift, filename="zap.ar").unload("zap.ar")
    plt.close("all")
    cleaner.clean(ica.Archive_load("zap.ar"), cleaner.parse_arguments(["-l", "-q", "-z", "zap.ar"]), "zap.ar")
    img = plt.imread("zap.ar_5_5.png")
    plt.close("all")
    assert img.shape == z["image"].shape and np.array_equal(img, z["image"])
