"""IR protocol specifications; tools/gen_ir.py generates their device and oracle forms."""
