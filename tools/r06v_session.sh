bash tools/gpu_session.sh r06ze "tests:entropy or stream or ac_run or gdec or jpeg or spec" htrace:fhd420_jpeg:product py:tools/fhd_ab.py:--variants,base,--rounds,3
