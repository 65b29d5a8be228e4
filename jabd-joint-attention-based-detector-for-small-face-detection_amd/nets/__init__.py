"""Drop-in replacements for the reference's `nets.*` modules (same class
names, constructor arguments and state_dict keys), whose forward passes run
on the MI355X HIP path (jabd_amd)."""
