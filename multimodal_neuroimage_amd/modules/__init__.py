"""Drop-in counterparts of the reference's modules/* (hot path on libmmni.so)."""
