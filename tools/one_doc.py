import os, sys
sys.path[:0] = ['language-detector_amd', 'oracle']
import cld_amd
from oracle import Oracle
d = open(sys.argv[1], 'rb').read()
cld_amd.init_device(0, tables=cld_amd.SYNTH_TABLES)
g = cld_amd.detect_batch(docs=[d])[0]
b, o = cld_amd.pack([d]); r = Oracle().detect_batch(b, o)[0]
print(os.environ.get('CLD_LONG_SPEC', '-'), 'gpu tb', g['text_bytes'], 'oracle tb', r['text_bytes'], flush=True)
