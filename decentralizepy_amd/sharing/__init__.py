"""Drop-in Sharing plugins (reference decentralizepy.sharing.*) backed by the HIP codec.

Select them from a decentralizepy config.ini exactly like the reference classes, e.g.::

    [SHARING]
    sharing_package = decentralizepy_amd.sharing.JWINS.JWINS
    sharing_class = JWINS
"""
